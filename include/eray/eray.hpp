// eray.hpp — the C++ host of the MI355X path: the reference's Scene / Graph builder API
// (src/lib) above the C-ABI of include/eray_hip.h.  Link liberay_host.so (+ liberay_hip.so).
#pragma once

#include "engine.hpp"
#include "graph.hpp"
#include "image.hpp"
#include "shaderlib.hpp"
