"""The wave node's cosf (eray_amd/csrc/glibc_cosf.hpp) is a restatement of the reference
platform's libm cosf (glibc 2.35: ARM optimized-routines sincosf).  Checked here on the host
(the same header is compiled for the GPU): bit-identical to the host glibc on a strided sweep
of all finite floats and on every argument main.rs's graph produces.  (A one-off exhaustive run
over all 4,278,190,080 finite floats found 0 mismatches.)"""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "eray_amd", "csrc", "glibc_cosf.hpp")

PROG = r"""
#include "%s"
#include <cstdio>
#include <cstdlib>
int main(int argc, char** argv) {
  unsigned step = (unsigned)strtoul(argv[1], 0, 10);
  long bad = 0, tot = 0;
  for (unsigned long long b = 0; b < 0x7f800000ULL; b += step)
    for (int s = 0; s < 2; ++s) {
      unsigned u = (unsigned)b | (s ? 0x80000000u : 0u); float a; memcpy(&a, &u, 4);
      float g = cosf(a), r = eray::libm::cosf_glibc(a); ++tot;
      if (eray::libm::f32_bits(g) != eray::libm::f32_bits(r)) ++bad;
    }
  // every argument of main.rs's wave node: (x + y) / 10 for x, y in 0..1024
  for (int k = 0; k <= 2046; ++k) { float a = (float)k / 10.0f; ++tot;
    if (eray::libm::f32_bits(cosf(a)) != eray::libm::f32_bits(eray::libm::cosf_glibc(a))) ++bad; }
  // specials
  float sp[] = {0.0f, -0.0f, __builtin_inff(), -__builtin_inff(), __builtin_nanf(""), 120.0f, 0x1p-12f};
  for (float a : sp) { ++tot; float g = cosf(a), r = eray::libm::cosf_glibc(a);
    if (!(g != g && r != r) && eray::libm::f32_bits(g) != eray::libm::f32_bits(r)) ++bad; }
  printf("%%ld %%ld\n", bad, tot);
  return 0;
}
"""


def test_cosf_matches_host_glibc(tmp_path):
    src = tmp_path / "c.cpp"
    src.write_text(PROG % HDR)
    exe = tmp_path / "c"
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-std=c++17", str(src), "-o", str(exe), "-lm"], check=True)
    out = subprocess.run([str(exe), "1009"], check=True, capture_output=True, text=True).stdout.split()
    bad, tot = int(out[0]), int(out[1])
    assert tot > 4_000_000
    assert bad == 0, f"{bad} of {tot} differ from glibc cosf"


DIV10_PROG = r"""
#include "%s"
#include <cstdio>
int main() {
  long bad = 0, fast = 0;
#pragma omp parallel for reduction(+:bad,fast) schedule(dynamic, 1)
  for (long hi = 0; hi < 256; ++hi)
    for (unsigned lo = 0; lo < (1u << 24); ++lo) {
      unsigned u = (unsigned)(hi << 24) | lo; float a; memcpy(&a, &u, 4);
      volatile float ten = 10.0f;
      const float g = a / ten, r = eray::libm::div10_f32(a);
      const unsigned e = (u >> 23) & 0xffu;
      if (e >= 32u && e <= 254u) ++fast;
      if (!(g != g && r != r) && eray::libm::f32_bits(g) != eray::libm::f32_bits(r)) ++bad;
    }
  printf("%%ld %%ld\n", bad, fast);
  return 0;
}
"""


def test_div10_is_the_ieee_quotient_for_every_float(tmp_path):
    """div10_f32 (the wave node's `/ 10.`) against the host's IEEE division, all 2^32 inputs."""
    src = tmp_path / "d.cpp"
    src.write_text(DIV10_PROG % HDR)
    exe = tmp_path / "d"
    subprocess.run(["g++", "-O2", "-fopenmp", "-ffp-contract=off", "-std=c++17", str(src), "-o", str(exe), "-lm"],
                   check=True)
    bad, fast = map(int, subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split())
    assert fast > 3_700_000_000  # the product-and-correction path covers all but the extremes
    assert bad == 0


def test_inv_pio4_table_is_four_over_pi():
    """The published 24-entry table holds 4/pi's bits in 32-bit windows advancing 8 bits per entry:
    the header keeps the string "24 zero bits, then 4/pi" as 32-bit words (inv_pio4_word)."""
    prec = 400
    one = 1 << prec

    def arctan_inv(x):
        total, term, x2, n, sign = 0, one // x, x * x, 1, 1
        while term:
            total += sign * (term // n)
            term //= x2
            n += 2
            sign = -sign
        return total

    pi = 4 * (4 * arctan_inv(5) - arctan_inv(239))
    bits = bin((4 << (2 * prec)) // pi)[2:]
    byts = [0, 0, 0] + [int(bits[i * 8:(i + 1) * 8], 2) for i in range(30)]
    want = [int.from_bytes(bytes(byts[4 * j:4 * j + 4]), "big") for j in range(7)]
    text = open(HDR).read()
    block = text[text.index("inline uint32_t inv_pio4_word"):]
    got = [int(h, 16) for h in re.findall(r"0x([0-9a-f]+)u", block)[:7]]
    assert got == want
    # the windows of the table's 24 entries (the published values, sliding 8 bits per entry)
    word = int("".join(f"{w:032b}" for w in got), 2)
    entries = [(word >> (7 * 32 - 32 - 8 * i)) & 0xFFFFFFFF for i in range(24)]
    assert entries[:4] == [0xa2, 0xa2f9, 0xa2f983, 0xa2f9836e] and entries[23] == 0x3c439041


# ----------------------------------------------------------------------------------- powf ---
POWF_HDR = os.path.join(ROOT, "eray_amd", "csrc", "glibc_powf.hpp")

POWF_PROG = r"""
#include "%s"
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
using namespace eray::libm;
static long bad = 0, tot = 0;
static void chk(float x, float y) {
  volatile float vy = y;  // no constant folding of the host call
  float g = powf(x, vy), r = powf_glibc(x, y); ++tot;
  if (std::isnan(g) && std::isnan(r)) return;
  if (f32_bits(g) != f32_bits(r)) ++bad;
}
int main(int argc, char** argv) {
  unsigned step = (unsigned)strtoul(argv[1], 0, 10);
  float ys[] = {1.0f, 2.0f, 0.5f, 3.0f, -1.0f, -2.5f, 10.0f, 100.0f, 0.1f, 1.0f / 3.0f, 7.25f, -0.5f,
                0.0f, -0.0f, INFINITY, -INFINITY, NAN, 127.5f, -149.0f, 1e-7f, 33.0f, 1e10f, -1e10f};
  for (float y : ys)
    for (unsigned long long b = 0; b < 0x80000000ULL; b += step) {
      chk(f32_from_bits((uint32_t)b), y);
      chk(f32_from_bits((uint32_t)b | 0x80000000u), y);
    }
  std::mt19937 rng(1);
  std::uniform_real_distribution<float> u01(0.0f, 1.0f), uy(-40.0f, 40.0f);
  for (int i = 0; i < 2000000; ++i) chk(u01(rng), u01(rng) * 64.0f);  // the specular term's range
  for (int i = 0; i < 2000000; ++i) chk(f32_from_bits(rng()), f32_from_bits(rng()));
  for (int i = 0; i < 1000000; ++i) chk(u01(rng) * 4.0f, uy(rng));
  // powf(x, 1) == x (the kernels' specialisation when no material has a specular power)
  long id_bad = 0;
  for (unsigned long long b = 0; b < 0x100000000ULL; b += step) {
    float x = f32_from_bits((uint32_t)b);
    volatile float one = 1.0f;
    if (!std::isnan(x) && f32_bits(powf(x, one)) != (uint32_t)b) ++id_bad;
  }
  printf("%%ld %%ld %%ld\n", bad, tot, id_bad);
  return 0;
}
"""


def test_powf_matches_host_glibc(tmp_path):
    """The restated glibc powf (the specular term, engine.rs:171,174) against the host glibc:
    23 exponents over a strided sweep of every float sign and magnitude, 5M random pairs, and
    powf(x, 1) == x over a strided sweep (a one-off exhaustive run over all 2^32 floats found
    no exception).  Checked with and without FMA contraction of the polynomials: identical."""
    src = tmp_path / "p.cpp"
    src.write_text(POWF_PROG % POWF_HDR)
    exe = tmp_path / "p"
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-std=c++17", str(src), "-o", str(exe), "-lm"], check=True)
    out = subprocess.run([str(exe), "1021"], check=True, capture_output=True, text=True).stdout.split()
    bad, tot, id_bad = int(out[0]), int(out[1]), int(out[2])
    assert tot > 50_000_000
    assert bad == 0, f"{bad} of {tot} differ from glibc powf"
    assert id_bad == 0


def test_powf_tables_are_the_host_libm_bytes():
    """The log2 (1/c, log2 c) and exp2 tables and polynomials of glibc_powf.hpp appear verbatim in
    the host's libm.so.6 (the powf data objects: 16 x 2 doubles + 5 coefficients; 32 words +
    shift + 3 coefficients)."""
    import struct
    libm = next((p for p in ("/lib/x86_64-linux-gnu/libm.so.6", "/usr/lib/x86_64-linux-gnu/libm.so.6")
                 if os.path.exists(p)), None)
    if libm is None:
        pytest.skip("no host libm.so.6")
    data = open(libm, "rb").read()
    text = open(POWF_HDR).read()
    log2_block = text[text.index("PowfLog2 kTab[16]"):text.index("return kTab;")]
    pairs = [float.fromhex(h) for h in re.findall(r"(-?0x[0-9a-f.]+p[+-]?\d+)", log2_block)]
    assert len(pairs) == 32
    poly = [float.fromhex(h) for h in ("0x1.27616c9496e0bp-2", "-0x1.71969a075c67ap-2", "0x1.ec70a6ca7baddp-2",
                                       "-0x1.7154748bef6c8p-1", "0x1.71547652ab82bp0")]
    for name in ("A0 = ", "A1 = ", "A2 = ", "A3 = ", "A4 = "):
        assert name in text
    assert struct.pack("<37d", *(pairs + poly)) in data
    exp_block = text[text.index("uint64_t kTab[32]"):]
    words = [int(h, 16) for h in re.findall(r"0x([0-9a-f]{16})ull", exp_block)[:32]]
    cpoly = [float.fromhex(h) for h in ("0x1.c6af84b912394p-5", "0x1.ebfce50fac4f3p-3", "0x1.62e42ff0c52d6p-1")]
    assert struct.pack("<32Q", *words) + struct.pack("<4d", float.fromhex("0x1.8p+47"), *cpoly) in data
