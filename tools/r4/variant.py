"""Measurement variants of the HIP library without measurement code in the product source.

Each variant is a list of (old, new) text substitutions applied to a copy of
fem-libraries_amd/csrc/femasm.hip; the copy is compiled to abl/libfemasm_<name>.so (bench with
FEMASM_LIB=abl/libfemasm_<name>.so). Timing-only variants compute wrong matrices.

usage: python tools/r4/variant.py NAME [NAME ...]      (build in parallel)
       python tools/r4/variant.py --list
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = os.path.join(ROOT, "fem-libraries_amd", "csrc", "femasm.hip")
OUT = os.path.join(ROOT, "abl")

# k_gather_lin (FIX = fixed-point / FP64 both): ablations keep the block arithmetic live
V = {
    # no LDS accumulate (the values feed a never-true store so the arithmetic stays)
    "lin_noadd": [(
        "                atomicAdd(reinterpret_cast<unsigned long long*>(ap + i * GD + kk), q);",
        "                if (q == 0x123456789ull) ap[i * GD + kk] = 1.0;"), (
        "              for (int kk = 0; kk < GD; ++kk) atomicAdd(ap + i * GD + kk, G[i][kk]);",
        "              for (int kk = 0; kk < GD; ++kk) if (G[i][kk] == 1.2345e-300) ap[i * GD + kk] = 1.0;")],
    # no chunk stores to HBM (every store offset past the range)
    "lin_nostore": [(
        "NT * u < lim ? base : OOB, 16 * NT * u,", "OOB, 16 * NT * u,"), (
        "(tid == 0 && h) ? 0 : OOB, 0, NTS);", "OOB, 0, NTS);"), (
        "(tid == 1 && tail) ? 8 * (nv - 1) : OOB, 0, NTS);", "OOB, 0, NTS);")],
    # per-phase clocks of k_gather_lin (s_memtime at the barriers, summed per wave in LDS, then over
    # the launch into the scratch line `dump`; block 0 prints the running totals at each launch start)
    "lin_timing": [(
        "  __shared__ int32_t s_id[RING];      // chunk id of iteration m at s_id[m % RING]\n  dv2* acc2 = reinterpret_cast<dv2*>(acc);\n  const int tid = threadIdx.x;",
        "  __shared__ int32_t s_id[RING];\n  dv2* acc2 = reinterpret_cast<dv2*>(acc);\n  const int tid = threadIdx.x;\n"
        "  __shared__ unsigned long long s_tm[NT / 64][16];\n"
        "  if (tid < NT / 4) s_tm[tid / 16][tid % 16] = 0ull;\n"
        "  unsigned long long* const tmo = reinterpret_cast<unsigned long long*>(dump);\n"
        "  if (blockIdx.x == 0 && tid == 0) printf(\"lin_timing %llu %llu %llu %llu %llu %llu %llu %llu %llu\\n\", tmo[0], tmo[1], tmo[2], tmo[3], tmo[4], tmo[5], tmo[6], tmo[7], tmo[8]);\n"
        "  unsigned long long t_prev = __builtin_amdgcn_s_memtime(), r_prev = __builtin_amdgcn_s_memrealtime();\n"
        "#define FA_T(i) { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); if ((tid & 63) == 0) atomicAdd(&s_tm[tid >> 6][i], t_ - t_prev); t_prev = t_; }\n"), (
        "    // the id of chunk k + AHEAD\n",
        "    FA_T(6);\n    { const unsigned long long r_ = __builtin_amdgcn_s_memrealtime(); if ((tid & 63) == 0) { atomicAdd(&s_tm[tid >> 6][7], 1ull); atomicAdd(&s_tm[tid >> 6][8], r_ - r_prev); } r_prev = r_; }\n    // the id of chunk k + AHEAD\n"), (
        "    __syncthreads();  // B1: the chunk is accumulated\n    // the exchanges at raised",
        "    FA_T(0);\n    __syncthreads();  // B1: the chunk is accumulated\n    FA_T(1);\n    // the exchanges at raised"), (
        "    if constexpr (FIX) {  // chunk k+1's scale",
        "    FA_T(3);\n    if constexpr (FIX) {  // chunk k+1's scale"), (
        "    if constexpr (FIX) {  // the integer sums back to doubles",
        "    __builtin_amdgcn_s_waitcnt(0xC07F);\n    FA_T(2);\n    if constexpr (FIX) {  // the integer sums back to doubles"), (
        "    __syncthreads();  // B3: the accumulator is clean for the next chunk's atomics\n    keep_vgprs(v, hv, tv);\n",
        "    FA_T(4);\n    __syncthreads();  // B3: the accumulator is clean for the next chunk's atomics\n    keep_vgprs(v, hv, tv);\n    FA_T(5);\n"), (
        "    cur = nxt;\n  }\n  if (bad) atomicOr(P.err, 1);\n}",
        "    cur = nxt;\n  }\n  if (bad) atomicOr(P.err, 1);\n  __syncthreads();\n"
        "  if (tid < 9) { unsigned long long t = 0; for (int w = 0; w < NT / 64; ++w) t += s_tm[w][tid]; atomicAdd(tmo + tid, t); }\n}")],
    # per-phase clocks of k_gather_neo (as lin_timing): items, next records + B1, drain, B3, bottom
    "neo_timing": [(
        "  static_assert(SW * NTH >= (MAXB * BS2 + 1) / 2 + 1, \"chunk_drain covers every pair\");\n",
        "  static_assert(SW * NTH >= (MAXB * BS2 + 1) / 2 + 1, \"chunk_drain covers every pair\");\n"
        "  __shared__ unsigned long long s_tm[4][16];\n"
        "  if (threadIdx.x < 64) s_tm[threadIdx.x / 16][threadIdx.x % 16] = 0ull;\n"
        "  unsigned long long* const tmo = reinterpret_cast<unsigned long long*>(dump);\n"
        "  if (blockIdx.x == 0 && threadIdx.x == 0) printf(\"neo_timing %llu %llu %llu %llu %llu %llu %llu\\n\", tmo[0], tmo[1], tmo[2], tmo[3], tmo[4], tmo[5], tmo[6]);\n"
        "  unsigned long long t_prev = __builtin_amdgcn_s_memtime(), r_prev = __builtin_amdgcn_s_memrealtime();\n"
        "#define FN_T(i) { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); if ((threadIdx.x & 63) == 0) atomicAdd(&s_tm[threadIdx.x >> 6][i], t_ - t_prev); t_prev = t_; }\n"), (
        "  for (int k = 0; d0.nb >= 0; ++k) {\n    unsigned int rn = 0u;",
        "  for (int k = 0; d0.nb >= 0; ++k) {\n    FN_T(4);\n"
        "    { const unsigned long long r_ = __builtin_amdgcn_s_memrealtime(); if ((threadIdx.x & 63) == 0) { atomicAdd(&s_tm[threadIdx.x >> 6][5], 1ull); atomicAdd(&s_tm[threadIdx.x >> 6][6], r_ - r_prev); } r_prev = r_; }\n"
        "    unsigned int rn = 0u;"), (
        "    // chunk k+1's records / slots / masks: the item registers are dead here, and these loads are\n",
        "    FN_T(0);\n    // chunk k+1's records / slots / masks: the item registers are dead here, and these loads are\n"), (
        "    __syncthreads();  // B1: the chunk is accumulated\n    fa_dv2 dv[SW];",
        "    __syncthreads();  // B1: the chunk is accumulated\n    FN_T(1);\n    fa_dv2 dv[SW];"), (
        "    __syncthreads();  // B3: the accumulator is clean for the next chunk's atomics\n    keep_vgprs(dv, dh, dt);\n    // chunk k + AHEAD's id",
        "    FN_T(2);\n    __syncthreads();  // B3: the accumulator is clean for the next chunk's atomics\n    keep_vgprs(dv, dh, dt);\n    FN_T(3);\n    // chunk k + AHEAD's id"), (
        "  if (bad) atomicOr(P.err, 1);\n}\n\n// ------------------------------------------------------------------------------ block-owner gather",
        "  if (bad) atomicOr(P.err, 1);\n  __syncthreads();\n  if (threadIdx.x < 7) { unsigned long long t = 0; for (int w = 0; w < 4; ++w) t += s_tm[w][threadIdx.x]; atomicAdd(tmo + threadIdx.x, t); }\n}\n\n// ------------------------------------------------------------------------------ block-owner gather")],
    # k_gather_neo ablations (timing only, wrong matrices; round 5): the phi-table reads replaced by a
    # per-lane register value, the mu-term table reads likewise, no LDS accumulate, no chunk stores
    "neo_nophi": [(
        "          for (int kk = 0; kk < GD; ++kk) pbq[kk] = pb[ql * GD + kk];",
        "          for (int kk = 0; kk < GD; ++kk) pbq[kk] = fake_phi + (double)(ql * GD + kk);"), (
        "  for (int t = tid; t < NP2; t += NTH) acc2[t] = dv2{0.0, 0.0};\n\n  const int32_t* __restrict__ eadj = P.eadj;",
        "  for (int t = tid; t < NP2; t += NTH) acc2[t] = dv2{0.0, 0.0};\n  const double fake_phi = P.tab[tid % 8];\n  const int32_t* __restrict__ eadj = P.eadj;")],
    "neo_noT": [(
        "          for (int t = 0; t < NT; ++t) dot = fma(cur.hd[t], Ta[b * NT + t], dot);",
        "          for (int t = 0; t < NT; ++t) dot = fma(cur.hd[t], fake_phi + (double)t, dot);"), (
        "  for (int t = tid; t < NP2; t += NTH) acc2[t] = dv2{0.0, 0.0};\n\n  const int32_t* __restrict__ eadj = P.eadj;",
        "  for (int t = tid; t < NP2; t += NTH) acc2[t] = dv2{0.0, 0.0};\n  const double fake_phi = P.tab[tid % 8];\n  const int32_t* __restrict__ eadj = P.eadj;")],
    "neo_noadd": [(
        "            for (int kk = 0; kk < GD; ++kk) atomicAdd(ap + i * GD + kk, K[i][kk]);\n        }\n      }\n    }\n    // chunk k+1's records",
        "            for (int kk = 0; kk < GD; ++kk) if (K[i][kk] == 1.2345e-300) ap[i * GD + kk] = 1.0;\n        }\n      }\n    }\n    // chunk k+1's records")],
    "neo_nostore": [(
        "    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, v[u]), rs, full ? 16 * j : OOB, 0, AUX);",
        "    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, v[u]), rs, OOB + 0 * full, 0, AUX);")],
    # (round 5) the item record loads: none (points faked from the cell index) / half (points 2, 3 copied
    # from points 0, 1)
    "neo_norec": [(
        "        const dv2 v = pp[k];\n        it.pt[ql][2 * k] = v.x;",
        "        const dv2 v = dv2{(double)c * 1e-9 + k, (double)ql + 0.5};\n        it.pt[ql][2 * k] = v.x;")],
    "neo_halfrec": [(
        "        const dv2 v = pp[k];\n        it.pt[ql][2 * k] = v.x;",
        "        const dv2 v = ql < 2 ? pp[k] : dv2{it.pt[ql - 2][2 * k], it.pt[ql - 2][2 * k + 1]};\n        it.pt[ql][2 * k] = v.x;")],
    "neo_nostore2": [(
        "    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, v[u]), rv, NT * u < lim ? base : OOB, 16 * NT * u, NTS);\n  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, hv), rv, (tid == 0 && h) ? 0 : OOB, 0, NTS);\n  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, tv), rv, (tid == 1 && tail) ? 8 * (nv - 1) : OOB, 0, NTS);\n}",
        "    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, v[u]), rv, OOB + 0 * lim, 16 * NT * u, NTS);\n  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, hv), rv, OOB, 0, NTS);\n  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, tv), rv, OOB + 0 * tail, 0, NTS);\n}")],
    # (round 5) a 38 KB accumulator for every gather (timing of k_gather_lin on E: larger chunks,
    # ~120 instead of ~96 entries of the 128 a workgroup's lanes hold)
    "lin38k": [("constexpr int FA_GATHER_LDS = 32768;", "constexpr int FA_GATHER_LDS = 38912;")],
    "lin36k": [("constexpr int FA_GATHER_LDS = 32768;", "constexpr int FA_GATHER_LDS = 36864;")],
    # the plan's alternating-path search: fewer rounds / shorter chains (round 5)
    "kr1": [("constexpr int kKempeRounds = 4;", "constexpr int kKempeRounds = 1;")],
    "kr2": [("constexpr int kKempeRounds = 4;", "constexpr int kKempeRounds = 2;")],
    "kl3": [("constexpr int kKempeLen = 6;", "constexpr int kKempeLen = 3;")],
    # neo_timing with the next chunk's record loads counted in "items" (applied after neo_timing)
    "neo_tload": [("    FN_T(0);\n    // chunk k+1's records / slots / masks: the item registers are dead here, and these loads are\n",
                   "    // chunk k+1's records / slots / masks: the item registers are dead here, and these loads are\n"),
                  ("    load_item(d1, pf1, cur);\n    __syncthreads();  // B1: the chunk is accumulated\n    FN_T(1);",
                   "    load_item(d1, pf1, cur);\n    FN_T(0);\n    __syncthreads();  // B1: the chunk is accumulated\n    FN_T(1);")],
    # per-phase clocks of k_hex_mfma (block 0's waves print their sums at exit): pre-MFMA phase, MFMA
    # loop, post-MFMA barrier + next-cell consume, block stores
    "hex_timing": [("  int par = 0;\n", "  int par = 0;\n  unsigned long long h_t[4] = {0, 0, 0, 0}, h_p = __builtin_amdgcn_s_memtime();\n"
                    "#define FH_T(i) { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); h_t[i] += t_ - h_p; h_p = t_; }\n"),
                   ("    load_ids(ci + 2 * G, gv2, nv2);\n    __syncthreads();\n", "    load_ids(ci + 2 * G, gv2, nv2);\n    __syncthreads();\n    FH_T(0);\n"),
                   ("    if constexpr (MODE == 2) __syncthreads();  // every wave is past its MFMA loop: phi is free\n",
                    "    FH_T(1);\n    if constexpr (MODE == 2) __syncthreads();  // every wave is past its MFMA loop: phi is free\n"),
                   ("    gv1 = gv2;\n    nv1 = nv2;\n#pragma unroll\n    for (int j = 0; j < TPW; ++j) {\n      int ta, tb;",
                    "    gv1 = gv2;\n    nv1 = nv2;\n    FH_T(2);\n#pragma unroll\n    for (int j = 0; j < TPW; ++j) {\n      int ta, tb;"),
                   ("    lam = lam_n;\n    mu = mu_n;\n  }\n}\n",
                    "    lam = lam_n;\n    mu = mu_n;\n    FH_T(3);\n  }\n  if (blockIdx.x < 2 && lane == 0) printf(\"hex_timing %d %d %llu %llu %llu %llu\\n\", (int)blockIdx.x, wave, h_t[0], h_t[1], h_t[2], h_t[3]);\n}\n")],
    # k_neo_records_m occupancy: 2 waves / SIMD (195 VGPRs) or 4 (128)
    "nr2": [("__global__ __launch_bounds__(256, 3) void k_neo_records_m(", "__global__ __launch_bounds__(256) void k_neo_records_m(")],
    "nr4": [("__global__ __launch_bounds__(256, 3) void k_neo_records_m(", "__global__ __launch_bounds__(256, 4) void k_neo_records_m(")],
    # k_gather_lin's chunk stores: cache policy bits of the buffer stores (2 = nt, the default)
    "nts0": [("      constexpr int OOB = 0x40000000, NTS = 2;  // nt\n      // one descriptor over the chunk's nv values",
              "      constexpr int OOB = 0x40000000, NTS = 0;  // nt\n      // one descriptor over the chunk's nv values")],
    "nts1": [("      constexpr int OOB = 0x40000000, NTS = 2;  // nt\n      // one descriptor over the chunk's nv values",
              "      constexpr int OOB = 0x40000000, NTS = 1;  // nt\n      // one descriptor over the chunk's nv values")],
    "nts3": [("      constexpr int OOB = 0x40000000, NTS = 2;  // nt\n      // one descriptor over the chunk's nv values",
              "      constexpr int OOB = 0x40000000, NTS = 3;  // nt\n      // one descriptor over the chunk's nv values")],
    # (round 6) every drain's store cache policy (k_gather_lin's inline drain and xchg_drain): plain / sc0 sc1
    "xnts0": [("constexpr int OOB = 0x40000000, NTS = 2;  // nt\n", "constexpr int OOB = 0x40000000, NTS = 0;  // nt\n")],
    "xnts3": [("constexpr int OOB = 0x40000000, NTS = 2;  // nt\n", "constexpr int OOB = 0x40000000, NTS = 3;  // nt\n")],
    # (round 6) k_gather_lin / k_gather_neo: an XCD whose eighth of the visiting sequence is used up takes
    # the next chunks of the other XCDs' eighths (work stealing at the tail, the eighths stay contiguous;
    # an eighth's length clipped at nchunks so an empty id is final). Measured E -0.5 %, not shipped:
    # DESIGN.md §4 (suite failures with it in the product library, unexplained)
    "steal": [(
        "  auto chunk_of = [&](unsigned int j) -> int32_t {\n"
        "    return (int32_t)(j < uper ? min((unsigned)xc * uper + j, unc) : unc);\n  };",
        "  auto len_of = [&](int x) -> unsigned int {\n"
        "    const unsigned int b = (unsigned)x * uper;\n"
        "    return b >= unc ? 0u : min(uper, unc - b);\n  };\n"
        "  auto chunk_of = [&](unsigned int j) -> int32_t {\n"
        "    if (j < len_of(xc)) return (int32_t)((unsigned)xc * uper + j);\n"
        "    for (int s = 1; s < 8; ++s) {\n"
        "      const int v = (xc + s) & 7;\n"
        "      const unsigned int lv = len_of(v);\n"
        "      unsigned int* const vc = reinterpret_cast<unsigned int*>(P.ctr) + 32 * v;\n"
        "      if (__hip_atomic_load(vc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= lv) continue;\n"
        "      const unsigned int r = atomicInc(vc, 0xFFFFFFFFu);\n"
        "      if (r < lv) return (int32_t)((unsigned)v * uper + r);\n"
        "    }\n"
        "    return (int32_t)unc;\n  };")],
    # (round 6) affine Q2 quadrilaterals through k_gather_lin: workgroups of 128 / 192 items (chunks of at
    # most that many whole entries; at 256 the 1023-block cap binds first, ~144 entries). Patterns of the
    # source before FA_Q2QUAD_NT (128, adopted): kept as the record of profiles/r6/q2quad_nt_ab.txt
    "q2quad_nt128": [("  return gd == 3 && nn == 4 ? FA_P1TET_NT : gd == 3 && nn == 10 ? FA_P2TET_NT : 256;",
                      "  return gd == 3 && nn == 4 ? FA_P1TET_NT : gd == 3 && nn == 10 ? FA_P2TET_NT : gd == 2 && nn == 9 ? 128 : 256;")],
    "q2quad_nt192": [("  return gd == 3 && nn == 4 ? FA_P1TET_NT : gd == 3 && nn == 10 ? FA_P2TET_NT : 256;",
                      "  return gd == 3 && nn == 4 ? FA_P1TET_NT : gd == 3 && nn == 10 ? FA_P2TET_NT : gd == 2 && nn == 9 ? 192 : 256;")],
    # ... and smaller accumulators (more resident workgroups): items per workgroup / blocks per chunk
    "q2quad_nt128_b767": [('  return gd == 3 && nn == 4 ? FA_P1TET_NT : gd == 3 && nn == 10 ? FA_P2TET_NT : 256;', '  return gd == 3 && nn == 4 ? FA_P1TET_NT : gd == 3 && nn == 10 ? FA_P2TET_NT : gd == 2 && nn == 9 ? 128 : 256;'), ('  return nn == gd + 1 ? kLinLdsP1 / (8 * gd * gd) : gather_maxb(false, gd * gd);', '  return nn == gd + 1 ? kLinLdsP1 / (8 * gd * gd) : gd == 2 && nn == 9 ? 767 : gather_maxb(false, gd * gd);')],
    "q2quad_nt128_b511": [('  return gd == 3 && nn == 4 ? FA_P1TET_NT : gd == 3 && nn == 10 ? FA_P2TET_NT : 256;', '  return gd == 3 && nn == 4 ? FA_P1TET_NT : gd == 3 && nn == 10 ? FA_P2TET_NT : gd == 2 && nn == 9 ? 128 : 256;'), ('  return nn == gd + 1 ? kLinLdsP1 / (8 * gd * gd) : gather_maxb(false, gd * gd);', '  return nn == gd + 1 ? kLinLdsP1 / (8 * gd * gd) : gd == 2 && nn == 9 ? 511 : gather_maxb(false, gd * gd);')],
    "q2quad_nt64_b511": [('  return gd == 3 && nn == 4 ? FA_P1TET_NT : gd == 3 && nn == 10 ? FA_P2TET_NT : 256;', '  return gd == 3 && nn == 4 ? FA_P1TET_NT : gd == 3 && nn == 10 ? FA_P2TET_NT : gd == 2 && nn == 9 ? 64 : 256;'), ('  return nn == gd + 1 ? kLinLdsP1 / (8 * gd * gd) : gather_maxb(false, gd * gd);', '  return nn == gd + 1 ? kLinLdsP1 / (8 * gd * gd) : gd == 2 && nn == 9 ? 511 : gather_maxb(false, gd * gd);')],
    "q2quad_nt64_b383": [('  return gd == 3 && nn == 4 ? FA_P1TET_NT : gd == 3 && nn == 10 ? FA_P2TET_NT : 256;', '  return gd == 3 && nn == 4 ? FA_P1TET_NT : gd == 3 && nn == 10 ? FA_P2TET_NT : gd == 2 && nn == 9 ? 64 : 256;'), ('  return nn == gd + 1 ? kLinLdsP1 / (8 * gd * gd) : gather_maxb(false, gd * gd);', '  return nn == gd + 1 ? kLinLdsP1 / (8 * gd * gd) : gd == 2 && nn == 9 ? 383 : gather_maxb(false, gd * gd);')],
    # (round 6) config E: a larger k_gather_lin accumulator for P2 tets (455 blocks = 32 KB; 4 workgroups
    # of ~40 KB still fit a CU's 160 KB): chunks fill more of their 128 entries
    "p2tet_b500": [('  return nn == gd + 1 ? kLinLdsP1 / (8 * gd * gd) : gather_maxb(false, gd * gd);', '  return nn == gd + 1 ? kLinLdsP1 / (8 * gd * gd) : gd == 3 && nn == 10 ? 500 : gather_maxb(false, gd * gd);'), ('  if (P.plan_maxb > gather_maxb(false, GD * GD))\n    return fail(FA_E_ARG, "gather plan chunks hold up to %d blocks, this form\'s kernel %d: plan with fa_plan_gather_form",\n                P.plan_maxb, gather_maxb(false, GD * GD));', '  if (P.plan_maxb > std::max(gather_maxb(false, GD * GD), lin_maxb(GD, NN)))\n    return fail(FA_E_ARG, "gather plan chunks hold up to %d blocks, this form\'s kernel %d: plan with fa_plan_gather_form",\n                P.plan_maxb, gather_maxb(false, GD * GD));')],
    "p2tet_b540": [('  return nn == gd + 1 ? kLinLdsP1 / (8 * gd * gd) : gather_maxb(false, gd * gd);', '  return nn == gd + 1 ? kLinLdsP1 / (8 * gd * gd) : gd == 3 && nn == 10 ? 540 : gather_maxb(false, gd * gd);'), ('  if (P.plan_maxb > gather_maxb(false, GD * GD))\n    return fail(FA_E_ARG, "gather plan chunks hold up to %d blocks, this form\'s kernel %d: plan with fa_plan_gather_form",\n                P.plan_maxb, gather_maxb(false, GD * GD));', '  if (P.plan_maxb > std::max(gather_maxb(false, GD * GD), lin_maxb(GD, NN)))\n    return fail(FA_E_ARG, "gather plan chunks hold up to %d blocks, this form\'s kernel %d: plan with fa_plan_gather_form",\n                P.plan_maxb, gather_maxb(false, GD * GD));')],
    # (round 6) config C: k_gather_lin P1-tet workgroups of 128 items (the Q2-quad lesson), accumulator 16 / 8 KB
    "p1tet_nt128": [('constexpr int FA_P1TET_NT = 256;', 'constexpr int FA_P1TET_NT = 128;')],
    "p1tet_nt128_lds8k": [('constexpr int FA_P1TET_NT = 256;', 'constexpr int FA_P1TET_NT = 128;'), ('constexpr int kLinLdsP1 = 16384;', 'constexpr int kLinLdsP1 = 8192;')],
    "p1tet_lds24k": [('constexpr int kLinLdsP1 = 16384;', 'constexpr int kLinLdsP1 = 24576;')],
    # (round 6) config E's set_diagonal pass: a smaller constrained-dof queue (LDS) per workgroup
    "bcq1024": [("constexpr int NT = 256, QCAP = 4096;", "constexpr int NT = 256, QCAP = 1024;")],
    "bcq512": [("constexpr int NT = 256, QCAP = 4096;", "constexpr int NT = 256, QCAP = 512;")],
    # the source as it is (A/B base of an edited product library)
    "base": [],
    # P1 simplices through the records kernel + k_gather_lin (no fused records)
    "nofuse": [("constexpr int FA_LIN_FUSE = 1;", "constexpr int FA_LIN_FUSE = 0;")],
    # k_gather_neo in 2-wave workgroups (128 items, chunks of <= 64 entries, 23 KB accumulator): 4
    # workgroups per CU instead of 2 (round 4 measured 77.2 vs 75.9 ms with the previous drain)
    "neo128": [("constexpr int FA_GATHER_LDS_NEO = 46080;", "constexpr int FA_GATHER_LDS_NEO = 23040;"),
               ("__launch_bounds__(256, 2) void k_gather_neo(", "__launch_bounds__(128, 2) void k_gather_neo("),
               ("  constexpr int NTH = 256;  // threads: 256 items", "  constexpr int NTH = 128;  // threads: 256 items"),
               ("                             256 / neo_nsplit(mesh->cell_type, mesh->degree));",
                "                             128 / neo_nsplit(mesh->cell_type, mesh->degree));"),
               ("gather_grid(k_gather_neo<GD, NN, NQ, NSPLIT>, P.nchunks, 256);\n    k_gather_neo<GD, NN, NQ, NSPLIT><<<(unsigned)grid, 256, 0, s>>>",
                "gather_grid(k_gather_neo<GD, NN, NQ, NSPLIT>, P.nchunks, 128);\n    k_gather_neo<GD, NN, NQ, NSPLIT><<<(unsigned)grid, 128, 0, s>>>")],
    # positional plans without the bank-balancing entry placement: position = adjacency order
    # (entries of a row, and of neighbouring rows, share cells: lanes of a quarter read nearby records)
    "perm_id": [("      const int j = gather_perm(jj, na, st, inv);\n      const int64_t e = a0 + j;\n      int64_t lo = r0, hi = r1 - 1;\n      while (lo < hi) {\n        const int64_t mid = (lo + hi + 1) >> 1;\n        if (adj_ptr[mid] <= e) lo = mid; else hi = mid - 1;\n      }\n      const int rowlo = (int)(indptr[lo] - b0);\n      uint8_t res[NN];",
                 "      const int j = jj;\n      const int64_t e = a0 + j;\n      int64_t lo = r0, hi = r1 - 1;\n      while (lo < hi) {\n        const int64_t mid = (lo + hi + 1) >> 1;\n        if (adj_ptr[mid] <= e) lo = mid; else hi = mid - 1;\n      }\n      const int rowlo = (int)(indptr[lo] - b0);\n      uint8_t res[NN];"),
                ("      const int pos = best * EQ + fill[best];", "      const int pos = jj;")],
    # the neo-Hookean gather with items of whole entries (10 columns, 256 per chunk) instead of 5 columns
    "neo1": [("constexpr int FA_GATHER_LDS_NEO = 46080;", "constexpr int FA_GATHER_LDS_NEO = 1022 * 72;"),
             ("constexpr int FA_NEO_NSPLIT = 2;", "constexpr int FA_NEO_NSPLIT = 1;")],
}


def subs(name):
    """a variant name, or several joined by '+' (applied in order)"""
    return [x for n in name.split("+") for x in V[n]]


def build(name):
    src = open(SRC).read()
    for old, new in subs(name):
        if old not in src:
            raise SystemExit(f"variant {name}: pattern not found:\n{old}")
        src = src.replace(old, new)
    os.makedirs(OUT, exist_ok=True)
    path = os.path.join(ROOT, "fem-libraries_amd", "csrc", f"_variant_{name}.hip")
    open(path, "w").write(src)
    return subprocess.Popen(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                             "-munsafe-fp-atomics", "-o", os.path.join(OUT, f"libfemasm_{name}.so"), path]), path


if __name__ == "__main__":
    if sys.argv[1:] == ["--list"]:
        print("\n".join(V))
        raise SystemExit(0)
    for n in sys.argv[1:]:  # every pattern checked (in order) before any build starts
        src = open(SRC).read()
        for old, new in subs(n):
            if old not in src:
                raise SystemExit(f"variant {n}: pattern not found:\n{old}")
            src = src.replace(old, new)
    procs = [build(n) for n in sys.argv[1:]]
    rc = 0
    for p, path in procs:
        rc |= p.wait()
        os.remove(path)
    raise SystemExit(rc)
