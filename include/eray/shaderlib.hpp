// shaderlib.hpp — the reference's src/shaderlib (wave, rgb, flat_color, mix_color): each
// module's node() (a GraphNode whose Shader runs the node operator on the GPU through the
// C-ABI), graph() (the node wrapped in a graph with defaults) and material(), plus main.rs's
// example material.
#pragma once

#include "engine.hpp"
#include "graph.hpp"

namespace eray {
namespace shaderlib {

using GraphResult = shader::Graph<shader::Unvalidated>;
using NodeResult = shader::Node<shader::Unvalidated>;

namespace wave {  // wave.rs
constexpr float DEFAULT_FACTOR = 1.0f;
NodeResult node();
shader::Status graph(GraphResult* out);
}  // namespace wave

namespace rgb {  // rgb.rs (the node's rgb.ppm debug dump is not reproduced)
NodeResult node();
shader::Status graph(GraphResult* out);
}  // namespace rgb

namespace flat_color {  // flat_color.rs
NodeResult node();
shader::Status graph(GraphResult* out);
}  // namespace flat_color

namespace mix_color {  // mix_color.rs
constexpr float DEFAULT_FACTOR = 0.5f;
NodeResult node();
shader::Status graph(GraphResult* out);
}  // namespace mix_color

// shaderlib/mod.rs elib(): the library as imported nodes
std::vector<shader::ImportedNode<shader::Unvalidated>> elib();

// main.rs:80-144: mix(rgb(wave, wave, wave), flat_color(r, g, b), factor); color <- mixer,
// diffuse <- wave
shader::Status example_material(Material* out);

}  // namespace shaderlib
}  // namespace eray
