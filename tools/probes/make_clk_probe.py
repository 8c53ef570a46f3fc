#!/usr/bin/env python3
"""Writes the s_memtime-instrumented crc32_kernels.hip that tools/probes/group_clocks.py reads
(class 0, the 2-lane group path): per wave, kernel entry / after the LDS fill / after the group
phase, and per round the descriptor wait (list entry -> len/off/crc_in -> the round's block count),
the chain (data loads, trailing bytes, blocks, tree), and the store. A probe build only (never
the product library):

  python tools/probes/make_clk_probe.py /tmp/k_probe.hip && tools/ab_build.sh /tmp/k_probe.hip clk0
  AMBRYCRC_LIBRARY=build/ab/clk0/libambrycrc.so python tools/probes/group_clocks.py batch100
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def sub(s, old, new):
    assert old in s, old[:70]
    return s.replace(old, new, 1)


def main(dst):
    s = open(os.path.join(ROOT, "ambry_amd", "csrc", "crc32_kernels.hip")).read()
    i = s.index("namespace ambrycrc {") + len("namespace ambrycrc {")
    s = s[:i] + "\n__device__ unsigned long long g_probe_clk[8192 * 8];\n" + s[i:]
    s = sub(s, "  fill_lds(a.img);\n\n  const uint32_t lane = threadIdx.x & 63u;",
            "  const uint64_t t_entry = clock64();\n  fill_lds(a.img);\n  const uint64_t t_fill = clock64();\n\n"
            "  const uint32_t lane = threadIdx.x & 63u;")
    grp = "    if (grp) group_phase_cls<true, COPY>(a, wave, nwaves, lane, make_lane_const(lane));\n"
    s = sub(s, grp, grp + "    if (!COPY && lane == 0 && wave < 8192) {\n      g_probe_clk[wave * 8 + 0] = t_entry;\n"
            "      g_probe_clk[wave * 8 + 1] = t_fill;\n      g_probe_clk[wave * 8 + 2] = clock64();\n    }\n")
    s = sub(s, "  const uint32_t gi = lane / G;\n#pragma unroll 1\n  for (uint64_t i = i0; i < i1; i += S) {\n"
               "    const bool act = i + gi < i1;",
            "  const uint32_t gi = lane / G;\n  uint64_t p_meta = 0, p_crc = 0, p_store = 0, p_rounds = 0;\n"
            "#pragma unroll 1\n  for (uint64_t i = i0; i < i1; i += S) {\n    const uint64_t t_a = clock64();\n"
            "    const bool act = i + gi < i1;")
    s = sub(s, "    const bool leader = (lane & (G - 1)) == 0 && act;\n    uint64_t stored = 0;",
            "    asm volatile(\"\" ::\"s\"(nbw));\n    const uint64_t t_b = clock64();\n"
            "    const bool leader = (lane & (G - 1)) == 0 && act;\n    uint64_t stored = 0;")
    s = sub(s, "    const uint32_t crc = group_crc_g<G, NB, NT, COPY>(a.base, off, len, cin, nbw, lane, k, dbase);\n"
               "    if (leader) {\n      a.out[ci] = crc;\n"
               "      if (a.exp_fill) a.exp_fill[ci] = (stored >> 32) ? ~crc : (uint32_t)stored;\n    }\n  }\n}",
            "    const uint32_t crc = group_crc_g<G, NB, NT, COPY>(a.base, off, len, cin, nbw, lane, k, dbase);\n"
            "    asm volatile(\"\" ::\"v\"(crc));\n    const uint64_t t_c = clock64();\n"
            "    if (leader) {\n      a.out[ci] = crc;\n"
            "      if (a.exp_fill) a.exp_fill[ci] = (stored >> 32) ? ~crc : (uint32_t)stored;\n    }\n"
            "    const uint64_t t_d = clock64();\n    p_meta += t_b - t_a;\n    p_crc += t_c - t_b;\n"
            "    p_store += t_d - t_c;\n    ++p_rounds;\n  }\n  if (lane == 0 && wave < 8192) {\n"
            "    g_probe_clk[wave * 8 + 4] += p_meta;\n    g_probe_clk[wave * 8 + 5] += p_crc;\n"
            "    g_probe_clk[wave * 8 + 6] += p_store;\n    g_probe_clk[wave * 8 + 7] += p_rounds;\n  }\n}")
    s += ("\nextern \"C\" int ambrycrc_probe_clocks(unsigned long long* out, size_t n) {\n"
          "  if (n > 8192 * 8) n = 8192 * 8;\n  return hipMemcpyFromSymbol(out, HIP_SYMBOL(ambrycrc::g_probe_clk), n * 8, 0,"
          " hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;\n}\n")
    open(dst, "w").write(s)


if __name__ == "__main__":
    main(sys.argv[1])
