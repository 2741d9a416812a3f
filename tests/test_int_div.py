"""The launch-invariant division of the shaderlib kernels' texel index (eray_amd/csrc/int_div.hpp,
Granlund & Montgomery 1994): equal to n / d on the host, exhaustively over every 32-bit n for a
few divisors and on a dense sample (every multiple of d and its neighbours) for the rest."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "eray_amd", "csrc", "int_div.hpp")

PROG = r"""
#include "%s"
#include <cstdio>
int main() {
  long bad = 0;
  const uint32_t full[] = {1u, 3u, 1024u, 1920u};
  for (uint32_t d : full) {
    const eray::DivU32 v = eray::make_div_u32(d);
#pragma omp parallel for reduction(+:bad) schedule(dynamic, 1)
    for (long hi = 0; hi < 256; ++hi)
      for (uint32_t lo = 0; lo < (1u << 24); ++lo) {
        const uint32_t n = (uint32_t)(hi << 24) | lo;
        if (eray::div_u32(n, v) != n / d) ++bad;
      }
  }
  const uint32_t some[] = {2u, 7u, 10u, 37u, 129u, 3840u, 7680u, 65535u, 65536u, 1000003u, 0x7fffffffu, 0x80000001u, 0xfffffffeu, 0xffffffffu};
  for (uint32_t d : some) {
    const eray::DivU32 v = eray::make_div_u32(d);
    for (uint64_t k = 0; k * d <= 0xffffffffull; k += (d < 4096 ? 997 : 1)) {
      for (int64_t e = -1; e <= 1; ++e) {
        const int64_t n = (int64_t)(k * d) + e;
        if (n < 0 || n > 0xffffffffll) continue;
        if (eray::div_u32((uint32_t)n, v) != (uint32_t)n / d) ++bad;
      }
    }
  }
  printf("%%ld\n", bad);
  return 0;
}
"""


def test_div_u32_equals_division(tmp_path):
    src = tmp_path / "d.cpp"
    src.write_text(PROG % HDR)
    exe = tmp_path / "d"
    subprocess.run(["g++", "-O2", "-fopenmp", "-std=c++17", str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()
    assert int(out[0]) == 0
