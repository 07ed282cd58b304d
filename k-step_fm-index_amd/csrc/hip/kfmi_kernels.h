/*
 * kfmi_kernels.h -- the search-side kernels and their launchers, shared by
 * kfmi_search.hip (host logic, dispatch) and the kfmi_inst_*.hip translation
 * units that instantiate dispatch_one<K, NB, LAY> for one (K, layout) each, so
 * the ~700 kernel instantiations compile in parallel.
 */
#ifndef KFMI_KERNELS_H_
#define KFMI_KERNELS_H_

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "kfmi_device.h"
#include "kfmi_grid.h"
#include "kfmi_coop.h"
#include "kfmi_locate.h"

namespace kfmi {

/* ------------------------------------------------------------------------ */
/* task-per-query kernel: one thread owns QPT queries (both ends each)       */
/* MAXW == 0: codes come from the pack kernel's words (qp);                 */
/* MAXW  > 0: the thread reads its own ASCII row once and keeps the codes   */
/*            in MAXW registers (fused packing, no pack launch, no qp).     */
/* ------------------------------------------------------------------------ */


/* Both ends' blocks of one step: block(L), and block(R) only when it differs. */
template <class G, int QPT>
__device__ __forceinline__ void fetch_ends(const IdxArgs& ix, const uint32_t (&L)[QPT], const uint32_t (&R)[QPT],
                                           const uint32_t (&c)[QPT], Blk<G> (&kl)[QPT], Blk<G> (&kr)[QPT])
{
#pragma unroll
  for (int i = 0; i < QPT; ++i) fetch_block<G>(ix, L[i] / (uint32_t) G::D, c[i], kl[i]);
#pragma unroll
  for (int i = 0; i < QPT; ++i) {
    const uint32_t br = R[i] / (uint32_t) G::D;
    if (br != kl[i].b) fetch_block<G>(ix, br, c[i], kr[i]);
    else kr[i] = kl[i];
  }
}

/* Issue-all-then-wait fetch for 32-byte, 16-byte-aligned plane blocks (K=2
 * d=64, K=1 d=128) with one u32 counter word: every load of both ends from ONE
 * asm block that sets exec per lane group and per condition (R only where its
 * block differs from L's, block b-1's planes only where line_local_prev chose
 * them), then a single vmcnt(0).  Written in C++ (fetch_ends) the compiler
 * copies block(L) into block(R) before R's loads issue -- a wait for L's
 * data -- so the two ends' lines are never in flight together.
 * A part no lane of a group needs (R where every R shares L's block, the
 * b-1 planes where no lane counts forward) is branched over.  Forms (the
 * SPLIT template value): 8 = one group, 7 = two 32-lane groups (32 pages per
 * instruction at most).  3 Gbase, 10M x 100 bp, against the C++ four-group
 * split (profiles/r03/sweep_r3n.jsonl): task (tag 101, 4.5 GB) 12.52 ->
 * 10.93 ms with 7 (four 16-lane groups: 11.28, removed in round 4; 8: 16.11
 * -- past the translation reach one group stalls); task-ac (tag 201, 3 GB) 11.47 ->
 * 9.51 (8: 9.79); task-mid 9.46 -> 9.40; 150 bp task-ac 17.01 -> 14.43,
 * task-mid 14.41 -> 14.34.  Issuing every part unconditionally, empty exec
 * or not, cost 15-19 % on task / task-ac (sweep_r3m.jsonl): an instruction
 * with no active lane still takes its issue slot.
 */
template <class G>
struct X4 {
  static constexpr bool OK = G::SMALL && G::BMW == 8 && G::BOFF % 4 == 0 && G::EW % 4 == 0;
};

#define KFMI_X4_BODY(T)                                      \
  "s_and_b64 exec, %[sv], %[gm]\n"                           \
  "global_load_dwordx4 %[l0], %[al], off\n"                  \
  "global_load_dwordx4 %[l1], %[al], off offset:16\n"        \
  "global_load_dword %[cl], %[acl], off\n"                   \
  KFMI_X4_PREV_L(T)                                          \
  "s_and_b64 exec, %[sv], %[gm]\n"                           \
  "s_and_b64 exec, exec, %[nr]\n"                            \
  KFMI_X4_SJ("r" T)                                          \
  "global_load_dwordx4 %[r0], %[ar], off\n"                  \
  "global_load_dwordx4 %[r1], %[ar], off offset:16\n"        \
  "global_load_dword %[cr], %[acr], off\n"                   \
  KFMI_X4_PREV_R(T)                                          \
  KFMI_X4_SL("r" T)
#define KFMI_X4_G1 "s_mov_b64 %[gm], -1\n" KFMI_X4_BODY("a")
#define KFMI_X4_G2 "s_bfm_b64 %[gm], 32, 0\n" KFMI_X4_BODY("a") "s_bfm_b64 %[gm], 32, 32\n" KFMI_X4_BODY("b")
#define KFMI_X4_ASM(GROUPS) "s_mov_b64 %[sv], exec\n" GROUPS "s_mov_b64 exec, %[sv]\ns_waitcnt vmcnt(0)\n"
#define KFMI_X4_OUT                                                                                          \
  [l0] "=&v"(l0), [l1] "=&v"(l1), [r0] "=&v"(r0), [r1] "=&v"(r1), [cl] "=&v"(cl), [cr] "=&v"(cr), [sv] "=&s"(sv), \
      [gm] "=&s"(gm)
#define KFMI_X4_IN [al] "v"(wl.planes), [acl] "v"(wl.cnt), [ar] "v"(wr.planes), [acr] "v"(wr.cnt), [nr] "s"(nr)
#define KFMI_X4_OUTP KFMI_X4_OUT, [p0] "=&v"(p0), [p1] "=&v"(p1), [q0] "=&v"(q0), [q1] "=&v"(q1)
#define KFMI_X4_INP KFMI_X4_IN, [pl] "s"(pl), [pr] "s"(pr), [po0] "i"(PO), [po1] "i"(PO + 16)
/* empty-exec skips: a branch over a part no lane of the group needs */
#define KFMI_X4_SJ(L) "s_cbranch_execz .Lx4" L "_%=\n"
#define KFMI_X4_SL(L) ".Lx4" L "_%=:\n"
#define KFMI_X4_PREV_L_ON(T)                                 \
  "s_and_b64 exec, exec, %[pl]\n"                            \
  KFMI_X4_SJ("p" T)                                          \
  "global_load_dwordx4 %[p0], %[al], off offset:%[po0]\n"    \
  "global_load_dwordx4 %[p1], %[al], off offset:%[po1]\n"    \
  KFMI_X4_SL("p" T)
#define KFMI_X4_PREV_R_ON(T)                                 \
  "s_and_b64 exec, exec, %[pr]\n"                            \
  KFMI_X4_SJ("r" T)                                          \
  "global_load_dwordx4 %[q0], %[ar], off offset:%[po0]\n"    \
  "global_load_dwordx4 %[q1], %[ar], off offset:%[po1]\n"

template <class G, int SPLIT>
__device__ __forceinline__ void fetch_ends_x4(const IdxArgs& ix, uint32_t L, uint32_t R, uint32_t c, Blk<G>& kl,
                                              Blk<G>& kr)
{
  static_assert(SPLIT == 7 || SPLIT == 8, "fetch form: 7, 8 = two, one lane group(s)");
  const uint32_t bl = L / (uint32_t) G::D, br = R / (uint32_t) G::D;
  Where<G> wl = locate<G>(ix, bl, c);
  Where<G> wr = locate<G>(ix, br, c);
  line_local_prev<G>(ix, bl, c, wl);
  line_local_prev<G>(ix, br, c, wr);
  const bool needR = br != bl;
  const uint64_t nr = __ballot(needR);
  v4u l0, l1, r0, r1;
  uint32_t cl, cr;
  uint64_t sv, gm;
  if constexpr (G::NEIGHBOR) {
    const uint64_t pl = __ballot(wl.prev), pr = __ballot(wr.prev);
    constexpr int PO = -4 * G::EW;   /* block b-1's planes, relative to block b's */
    v4u p0, p1, q0, q1;
#define KFMI_X4_PREV_L(T) KFMI_X4_PREV_L_ON(T)
#define KFMI_X4_PREV_R(T) KFMI_X4_PREV_R_ON(T)
    if constexpr (SPLIT == 8)
      asm volatile(KFMI_X4_ASM(KFMI_X4_G1) : KFMI_X4_OUTP : KFMI_X4_INP : "memory", "scc");
    else
      asm volatile(KFMI_X4_ASM(KFMI_X4_G2) : KFMI_X4_OUTP : KFMI_X4_INP : "memory", "scc");
#undef KFMI_X4_PREV_L
#undef KFMI_X4_PREV_R
    const v4u pa = needR ? q0 : p0, pb = needR ? q1 : p1;
    kl.bp[0] = p0.x; kl.bp[1] = p0.y; kl.bp[2] = p0.z; kl.bp[3] = p0.w;
    kl.bp[4] = p1.x; kl.bp[5] = p1.y; kl.bp[6] = p1.z; kl.bp[7] = p1.w;
    kr.bp[0] = pa.x; kr.bp[1] = pa.y; kr.bp[2] = pa.z; kr.bp[3] = pa.w;
    kr.bp[4] = pb.x; kr.bp[5] = pb.y; kr.bp[6] = pb.z; kr.bp[7] = pb.w;
  } else {
#define KFMI_X4_PREV_L(T)
#define KFMI_X4_PREV_R(T)
    if constexpr (SPLIT == 8)
      asm volatile(KFMI_X4_ASM(KFMI_X4_G1) : KFMI_X4_OUT : KFMI_X4_IN : "memory", "scc");
    else
      asm volatile(KFMI_X4_ASM(KFMI_X4_G2) : KFMI_X4_OUT : KFMI_X4_IN : "memory", "scc");
#undef KFMI_X4_PREV_L
#undef KFMI_X4_PREV_R
  }
  const v4u ra = needR ? r0 : l0, rb = needR ? r1 : l1;
  kl.bm[0] = l0.x; kl.bm[1] = l0.y; kl.bm[2] = l0.z; kl.bm[3] = l0.w;
  kl.bm[4] = l1.x; kl.bm[5] = l1.y; kl.bm[6] = l1.z; kl.bm[7] = l1.w;
  kr.bm[0] = ra.x; kr.bm[1] = ra.y; kr.bm[2] = ra.z; kr.bm[3] = ra.w;
  kr.bm[4] = rb.x; kr.bm[5] = rb.y; kr.bm[6] = rb.z; kr.bm[7] = rb.w;
  kl.cnt = cl;
  kr.cnt = needR ? cr : cl;
  kl.b = bl;
  kr.b = br;
  kl.e = wl.e;
  kr.e = wr.e;
  kl.prev = wl.prev;
  kr.prev = wr.prev;
}
#undef KFMI_X4_BODY
#undef KFMI_X4_G1
#undef KFMI_X4_G2
#undef KFMI_X4_ASM
#undef KFMI_X4_OUT
#undef KFMI_X4_IN
#undef KFMI_X4_OUTP
#undef KFMI_X4_INP
#undef KFMI_X4_SJ
#undef KFMI_X4_SL
#undef KFMI_X4_PREV_L_ON
#undef KFMI_X4_PREV_R_ON

/* The fetch forms (the SPLIT template value, launch_task): 1 = the C++ fetch
 * in one group; 4 = the same loads as four exec-masked 16-lane groups, so one
 * wave instruction touches at most 16 pages (IdxArgs::split); 7 / 8 = the asm
 * fetch in two / one group(s) (X4 geometries only). */
template <class G, int QPT, int SPLIT>
__device__ __forceinline__ void fetch_ends_split(const IdxArgs& ix, const uint32_t (&L)[QPT],
                                                 const uint32_t (&R)[QPT], const uint32_t (&c)[QPT],
                                                 Blk<G> (&kl)[QPT], Blk<G> (&kr)[QPT])
{
  static_assert(SPLIT == 1 || SPLIT == 4 || ((SPLIT == 7 || SPLIT == 8) && QPT == 1 && X4<G>::OK),
                "fetch form: 1 / 4 (C++ fetch), 7 / 8 (asm fetch, X4 geometries)");
  if constexpr (SPLIT >= 7) {
    fetch_ends_x4<G, SPLIT>(ix, L[0], R[0], c[0], kl[0], kr[0]);
  } else if constexpr (SPLIT == 1) {
    fetch_ends<G, QPT>(ix, L, R, c, kl, kr);
  } else {
    const int grp = (int) (threadIdx.x & 63) / 16;
#pragma unroll
    for (int g = 0; g < 4; ++g)
      if (grp == g) fetch_ends<G, QPT>(ix, L, R, c, kl, kr);
  }
}

template <class G, int QPT, int MAXW, int SPLIT = 1>
__global__ __launch_bounds__(256) void task_kernel(IdxArgs ix, const uint32_t* __restrict__ qp,
                                                   const uint8_t* __restrict__ ascii, uint32_t m, uint64_t num,
                                                   uint32_t steps, uint32_t nwords, uint32_t* __restrict__ res)
{
  constexpr int SPW = G::SPW;
  constexpr int CW = MAXW > 0 ? (G::K == 3 ? k3_words<(MAXW > 0 ? MAXW : 1)>() : MAXW) : 1;
  static_assert(MAXW == 0 || QPT == 1, "fused packing: one query per thread");
  const uint64_t base = (uint64_t) blockIdx.x * (256 * QPT) + threadIdx.x;
  uint32_t cw[QPT][CW];
  uint32_t rc = 0;
  if constexpr (MAXW > 0) {
    extern __shared__ __attribute__((aligned(16))) uint8_t stage[];
    if constexpr (G::K == 3) {   /* 16 bases per word -> 5 K-steps per word */
      uint32_t raw[MAXW];
      stage_query_codes<MAXW>(ascii, num, m, stage, raw, ix.rem, rc);   /* whole block, before any exit */
      recut30<MAXW>(raw, cw[0]);
    } else {
      stage_query_codes<MAXW>(ascii, num, m, stage, cw[0], ix.rem, rc);   /* whole block, before any exit */
    }
  }
  if (base >= num) return;
  uint64_t q[QPT];
  uint32_t L[QPT], R[QPT];
#pragma unroll
  for (int i = 0; i < QPT; ++i) {
    q[i] = base + (uint64_t) i * 256;
    if (q[i] >= num) q[i] = base;   /* duplicate work for the tail, never stored twice */
    L[i] = 0;
    R[i] = ix.bwtsize;
  }
  uint32_t skip = 0;
  if (ix.ftab && steps >= ix.ftab_steps) {   /* wave-uniform: jump start from the ftab */
    skip = ix.ftab_steps;
#pragma unroll
    for (int i = 0; i < QPT; ++i) {
      uint32_t w0;
      if constexpr (MAXW > 0) w0 = cw[i][0];
      else w0 = qp[q[i]];
      const uint2 lr = ix.ftab[w0 & ix.ftab_mask];
      L[i] = lr.x;
      R[i] = lr.y;
    }
  }
  if (ix.rem) {   /* wave-uniform: m % K != 0, the last rem bases from the remainder table */
#pragma unroll
    for (int i = 0; i < QPT; ++i) {
      const uint2 lr = ix.rtab[MAXW > 0 ? rc : qp[(uint64_t) nwords * num + q[i]]];
      L[i] = lr.x;
      R[i] = lr.y;
    }
  }
  for (uint32_t w = 0; w < nwords; ++w) {
    uint32_t word[QPT];
#pragma unroll
    for (int i = 0; i < QPT; ++i) {
      if constexpr (MAXW > 0) {
        word[i] = cw[i][0];
#pragma unroll
        for (int k = 0; k + 1 < CW; ++k) cw[i][k] = cw[i][k + 1];
      } else {
        word[i] = qp[(uint64_t) w * num + q[i]];
      }
    }
    const uint32_t left = steps - w * SPW;
#pragma unroll
    for (int j = 0; j < SPW; ++j) {
      if ((uint32_t) j >= left) continue;   /* only the last word is partial (wave-uniform) */
      if (w * SPW + j < skip) continue;      /* steps covered by the ftab (wave-uniform) */
      uint32_t c[QPT];
#pragma unroll
      for (int i = 0; i < QPT; ++i) c[i] = (word[i] >> (2 * G::K * j)) & (uint32_t) (G::NC - 1);
      if constexpr (G::SMALL) {
        Blk<G> kl[QPT], kr[QPT];
        fetch_ends_split<G, QPT, SPLIT>(ix, L, R, c, kl, kr);
#pragma unroll
        for (int i = 0; i < QPT; ++i) {
          uint32_t sx[2 * G::K];
          plane_xor<G::K>(c[i], sx);
          L[i] = lf_from_block<G>(ix, kl[i], L[i], c[i], sx);
          R[i] = lf_from_block<G>(ix, kr[i], R[i], c[i], sx);
        }
      } else {
#pragma unroll
        for (int i = 0; i < QPT; ++i) {
          uint32_t sx[2 * G::K];
          plane_xor<G::K>(c[i], sx);
          L[i] = lf_stream<G>(ix, L[i], c[i], sx);
          R[i] = lf_stream<G>(ix, R[i], c[i], sx);
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < QPT; ++i) {
    const uint64_t qi = base + (uint64_t) i * 256;
    if (qi < num) *reinterpret_cast<uint2*>(res + 2 * qi) = make_uint2(L[i], R[i]);
  }
}

/* ftab construction: [L, R) of every code stream v of ftab_steps K-steps
 * (the search's own first steps, from [0, n+1)), each end by lf_stream --
 * the per-row step of every non-search kernel.  Round 5 detoured this build
 * through the task kernels' fetch when lf_stream's K = 1, d = 64 AltCounters
 * form returned wrong entries; the cause was the 16-byte load at 8-byte
 * alignment LLVM formed from two 8-byte plane loads, which
 * load_words now keeps out, so the build is lf_stream's again and
 * test_ftab_table_every_entry checks its tables entry by entry. */
template <class G>
__global__ __launch_bounds__(256) void ftab_build_kernel(IdxArgs ix, uint32_t fsteps, uint64_t n,
                                                         uint2* __restrict__ out)
{
  /* grid-stride: 4^16 entries exceed the 2^32 work-items of one dispatch */
  for (uint64_t v = (uint64_t) blockIdx.x * 256 + threadIdx.x; v < n; v += (uint64_t) gridDim.x * 256) {
    uint32_t L = 0, R = ix.bwtsize;
    for (uint32_t t = 0; t < fsteps; ++t) {
      const uint32_t c = (uint32_t) (v >> (2 * G::K * t)) & (uint32_t) (G::NC - 1);
      uint32_t sx[2 * G::K];
      plane_xor<G::K>(c, sx);
      L = lf_stream<G>(ix, L, c, sx);
      R = lf_stream<G>(ix, R, c, sx);
    }
    out[v] = make_uint2(L, R);
  }
}

/* Remainder table for reads with m % K = rem (1 <= rem < K): [L, R) of every
 * rem-base string x (base m-1 at bits 0-1, the code order of the K-steps).
 * A K-step from [0, n+1) gives the suffix-array range of a K-mer, so
 *   R(x) = R of x.T^(K-rem)  (the last K-mer range inside x's),
 *   L(x) = L of x.A^(K-rem) - #{j < K-rem : T ends with x.A^j}
 * (the suffixes x.A^j.$ sort below x.A^(K-rem) but inside x's range).  Whether
 * T ends with x.A^j is read from row 0 (suffix "$"), whose K-mer code holds
 * T[n-1-s] at bits 2s.  One thread per x (4^rem <= 64). */
template <class G>
__global__ __launch_bounds__(64) void rem_tab_kernel(IdxArgs ix, uint32_t rem, uint2* __restrict__ out)
{
  const uint32_t x = threadIdx.x;
  if (rem == 0 || rem >= (uint32_t) G::K || x >= (1u << (2 * rem))) return;
  const uint32_t pad = 2 * ((uint32_t) G::K - rem);
  const uint32_t cA = x << pad, cT = cA | ((1u << pad) - 1u);
  uint32_t sx[2 * G::K];
  plane_xor<G::K>(cA, sx);
  uint32_t L = lf_stream<G>(ix, 0u, cA, sx);
  plane_xor<G::K>(cT, sx);
  const uint32_t R = lf_stream<G>(ix, ix.bwtsize, cT, sx);
  const uint32_t n = ix.bwtsize - 1u;
  const uint32_t tail = row_code<G>(ix, 0u);
  for (uint32_t j = 0; j + rem < (uint32_t) G::K; ++j)
    if (j + rem <= n && (tail & ((1u << (2 * j)) - 1u)) == 0u && ((tail >> (2 * j)) & ((1u << (2 * rem)) - 1u)) == x)
      --L;
  out[x] = make_uint2(L, R);
}

/* distinct d-blocks touched per step (1 if L/d == R/d else 2): the
 * dedup-aware algorithmic traffic of SURVEY 8(d).  Same LF math as the
 * task kernel; a separate launch so the timed kernels carry no counters. */
template <class G>
__global__ __launch_bounds__(256) void count_blocks_kernel(IdxArgs ix, const uint32_t* __restrict__ qp, uint64_t num,
                                                           uint32_t steps, uint32_t nwords,
                                                           unsigned long long* __restrict__ total)
{
  const uint64_t q = (uint64_t) blockIdx.x * 256 + threadIdx.x;
  uint32_t cnt = 0;
  if (q < num) {
    uint32_t L = 0, R = ix.bwtsize;
    if (ix.rem) {   /* a table lookup, no index line */
      const uint2 lr = ix.rtab[qp[(uint64_t) nwords * num + q]];
      L = lr.x;
      R = lr.y;
    }
    for (uint32_t t = 0; t < steps; ++t) {
      const uint32_t word = qp[(uint64_t) (t / G::SPW) * num + q];
      const uint32_t c = (word >> (2 * G::K * (t % G::SPW))) & (uint32_t) (G::NC - 1);
      uint32_t sx[2 * G::K];
      plane_xor<G::K>(c, sx);
      cnt += (L / (uint32_t) G::D == R / (uint32_t) G::D) ? 1u : 2u;
      L = lf_stream<G>(ix, L, c, sx);
      R = lf_stream<G>(ix, R, c, sx);
    }
  }
  /* wave reduction, one atomic per wave */
  for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off);
  if ((threadIdx.x & 63) == 0) atomicAdd(total, (unsigned long long) cnt);
}

/* Derivation of a 2K-step index from a K-step one (kfmi_derive_index_gpu):
 * row i's 2K-mer code is its own K-mer code (T[p-1-s], s < K, p = SA[i]) and,
 * above it, the K-mer code of row LF_K(i) -- the row of suffix p - K, whose
 * K-mer is T[p-1-K-s].  One thread per row (grid-stride).  The K rows whose
 * K-mer holds the '$' (D_s, s < K) have no valid LF: their upper half is
 * written by the host from the text's tail (row 0's code, see the caller);
 * a row whose LF lands on D_s is the row of suffix K + s, the new D_{K+s}
 * (isa[s]). */
/* The LF_K successor of every row for the walk check (check_lf_walks,
 * kfmi_search.hip): next[X] = LF_K(X) as a locate walk takes it (lf_row), a
 * '$' row D_s its own successor; an image past the last row sets *bad. */
template <class G>
__global__ __launch_bounds__(256) void lf_next_kernel(IdxArgs ix, uint64_t rows, uint32_t* __restrict__ next,
                                                      uint32_t* __restrict__ bad)
{
  for (uint64_t i = (uint64_t) blockIdx.x * 256 + threadIdx.x; i < rows; i += (uint64_t) gridDim.x * 256) {
    const uint32_t X = (uint32_t) i;
    bool dollar = false;
#pragma unroll
    for (int s = 0; s < G::K; ++s) dollar = dollar || ix.dl.dpos[s] == X;
    uint32_t j = X;
    if (!dollar) {
      j = lf_row<G>(ix, X);
      if ((uint64_t) j >= rows) {
        atomicOr(bad, 1u);
        j = X;
      }
    }
    next[i] = j;
  }
}

template <class G>
__global__ __launch_bounds__(256) void derive_codes_kernel(IdxArgs ix, uint64_t rows, uint8_t* __restrict__ codes,
                                                           uint32_t* __restrict__ isa)
{
  for (uint64_t i = (uint64_t) blockIdx.x * 256 + threadIdx.x; i < rows; i += (uint64_t) gridDim.x * 256) {
    const uint32_t X = (uint32_t) i;
    const uint32_t c = row_code<G>(ix, X);
    bool dollar = false;
#pragma unroll
    for (int s = 0; s < G::K; ++s) dollar = dollar || ix.dl.dpos[s] == X;
    uint32_t up = 0;
    if (!dollar) {
      uint32_t sx[2 * G::K];
      plane_xor<G::K>(c, sx);
      const uint32_t j = lf_stream<G>(ix, X, c, sx);
      up = row_code<G>(ix, j);
#pragma unroll
      for (int s = 0; s < G::K; ++s)
        if (ix.dl.dpos[s] == j) isa[s] = X;
    }
    codes[i] = (uint8_t) (c | (up << (2 * G::K)));
  }
}

/* 128-B lines one LF end's task-kernel fetch touches (fetch_block: the
 * planes, the counter word and, when the
 * step is counted forward from block b-1 (line_local_prev), b-1's planes).
 * Returns how many ids it appended to ln; *extra = 1 when the counter lies
 * outside the planes' line(s), *prev = 1 for a line-local step. */
template <class G>
__device__ __forceinline__ int lf_lines(const IdxArgs& ix, uint32_t X, uint32_t c, uint64_t* ln, uint32_t* extra,
                                        uint32_t* prev)
{
  const uint32_t b = X / (uint32_t) G::D;
  Where<G> w = locate<G>(ix, b, c);
  line_local_prev<G>(ix, b, c, w);
  int n = 0;
  const uint64_t p0 = (uint64_t) (uintptr_t) w.planes >> 7, p1 = (uint64_t) (uintptr_t) (w.planes + G::BMW - 1) >> 7;
  ln[n++] = p0;
  if (p1 != p0) ln[n++] = p1;
  const uint64_t cl = (uint64_t) (uintptr_t) w.cnt >> 7;
  *extra = (cl != p0 && cl != p1) ? 1u : 0u;
  if (*extra) ln[n++] = cl;
  *prev = w.prev ? 1u : 0u;
  if (w.prev) {
    const uint64_t q0 = (uint64_t) (uintptr_t) w.pplanes >> 7, q1 = (uint64_t) (uintptr_t) (w.pplanes + G::BMW - 1) >> 7;
    if (q0 != p0 && q0 != p1) ln[n++] = q0;
    if (q1 != q0 && q1 != p0 && q1 != p1) ln[n++] = q1;
  }
  return n;
}

/* Statistics only (not timed): per batch, the distinct 128-B lines each
 * K-step's fetches touch (L's block, and R's when it is another block, as the
 * task kernel fetches them; lines shared by the two ends counted once) --
 * out[0]; the ends whose counter lies outside their planes' line -- out[1];
 * the ends fetched -- out[2]; the ends counted forward from block b-1
 * (line-local) -- out[3].  Compared with the PMC's fabric requests per read
 * this splits a layout's requests into the structural lines its fetches need
 * and what the caches absorb. */
template <class G>
__global__ __launch_bounds__(256) void count_lines_kernel(IdxArgs ix, const uint32_t* __restrict__ qp, uint64_t num,
                                                          uint32_t steps, uint32_t nwords,
                                                          unsigned long long* __restrict__ out)
{
  const uint64_t q = (uint64_t) blockIdx.x * 256 + threadIdx.x;
  uint32_t lines = 0, extra = 0, ends = 0, prevs = 0;
  if (q < num) {
    uint32_t L = 0, R = ix.bwtsize;
    if (ix.rem) {
      const uint2 lr = ix.rtab[qp[(uint64_t) nwords * num + q]];
      L = lr.x;
      R = lr.y;
    }
    for (uint32_t t = 0; t < steps; ++t) {
      const uint32_t word = qp[(uint64_t) (t / G::SPW) * num + q];
      const uint32_t c = (word >> (2 * G::K * (t % G::SPW))) & (uint32_t) (G::NC - 1);
      uint64_t ln[10];
      uint32_t ex, pv;
      int n = lf_lines<G>(ix, L, c, ln, &ex, &pv);
      extra += ex;
      prevs += pv;
      ++ends;
      if (R / (uint32_t) G::D != L / (uint32_t) G::D) {
        n += lf_lines<G>(ix, R, c, ln + n, &ex, &pv);
        extra += ex;
        prevs += pv;
        ++ends;
      }
      for (int i = 0; i < n; ++i) {
        bool dup = false;
        for (int j = 0; j < i; ++j) dup = dup || ln[j] == ln[i];
        lines += dup ? 0u : 1u;
      }
      uint32_t sx[2 * G::K];
      plane_xor<G::K>(c, sx);
      L = lf_stream<G>(ix, L, c, sx);
      R = lf_stream<G>(ix, R, c, sx);
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    lines += __shfl_xor(lines, off);
    extra += __shfl_xor(extra, off);
    ends += __shfl_xor(ends, off);
    prevs += __shfl_xor(prevs, off);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(out + 0, (unsigned long long) lines);
    atomicAdd(out + 1, (unsigned long long) extra);
    atomicAdd(out + 2, (unsigned long long) ends);
    atomicAdd(out + 3, (unsigned long long) prevs);
  }
}

/* ------------------------------------------------------------------------ */
/* dispatch tables                                                          */
/* ------------------------------------------------------------------------ */

struct SearchLaunch {
  hipStream_t st;
  IdxArgs ix;
  const uint32_t* qp;
  const uint8_t* ascii;   /* fused packing: ASCII rows of m bases */
  uint32_t m;
  int maxw;               /* 0: packed words in qp; 8/16: fused packing */
  uint64_t num;
  uint32_t steps, nwords;
  uint32_t* res;
  /* locate */
  const uint32_t* sa;
  uint32_t sa_log2;
  const uint64_t* off;
  const uint32_t* owner;
  uint64_t total;
  uint32_t* pos;
  unsigned long long* slot_ctr;   /* walk slot queue, zeroed before the launch */
  uint32_t slot_chunk;            /* slots per queue take (64 .. 4096) */
  /* ftab build */
  uint2* ftab_out;
  uint32_t ftab_steps;
  uint64_t ftab_n;
  /* remainder table build: rem bases -> ftab_out */
  uint32_t rem;
  /* index derivation: 2K-mer code per row (num rows), the rows of suffixes K..2K-1 */
  uint8_t* derive_codes;
  uint32_t* derive_isa;
  /* walk check (Op::PermCheck): every row's LF_K successor, and the flag of an image past the rows */
  uint32_t* perm_next;
  uint32_t* perm_bad;
};

template <class G, int SPLIT>
static void launch_task_split(const SearchLaunch& a)
{
  if (a.maxw) {
    const uint64_t blocks = (a.num + 255) / 256;
    const size_t lds = 4 * (size_t) stage_slot_bytes(a.m);
    if (a.maxw == 8)
      hipLaunchKernelGGL((task_kernel<G, 1, 8, SPLIT>), dim3((uint32_t) blocks), dim3(256), lds, a.st, a.ix, a.qp,
                         a.ascii, a.m, a.num, a.steps, a.nwords, a.res);
    else
      hipLaunchKernelGGL((task_kernel<G, 1, 16, SPLIT>), dim3((uint32_t) blocks), dim3(256), lds, a.st, a.ix, a.qp,
                         a.ascii, a.m, a.num, a.steps, a.nwords, a.res);
  } else {
    const uint64_t blocks = (a.num + 255) / 256;
    hipLaunchKernelGGL((task_kernel<G, 1, 0, SPLIT>), dim3((uint32_t) blocks), dim3(256), 0, a.st, a.ix, a.qp,
                       a.ascii, a.m, a.num, a.steps, a.nwords, a.res);
  }
}

template <class G>
static hipError_t launch_task(const SearchLaunch& a)
{
  /* the split only exists for the one-line-per-block path (d <= 128 at K=2);
   * one fetch form per (geometry, table size class): the asm fetch in one group
   * below 2 GB, two groups above (X4 geometries); else the C++ fetch, in four
   * groups where split_for asks for them */
  if constexpr (G::SMALL) {
    const uint32_t want = a.ix.split;
    if constexpr (X4<G>::OK) {
      if (want == 1) launch_task_split<G, 8>(a);
      else launch_task_split<G, 7>(a);
      return hipGetLastError();
    }
    if (want == 4 || (want == 2 && a.maxw == 8)) {
      launch_task_split<G, 4>(a);
      return hipGetLastError();
    }
  }
  launch_task_split<G, 1>(a);
  return hipGetLastError();
}

template <class G>
static hipError_t launch_coop(const SearchLaunch& a)
{
  return coop_launch<G>(a.st, a.ix, a.qp, a.ascii, a.m, a.maxw, a.num, a.steps, a.nwords, a.res);
}

template <class G>
static hipError_t launch_count(const SearchLaunch& a, unsigned long long* d_total)
{
  const uint64_t blocks = (a.num + 255) / 256;
  hipLaunchKernelGGL((count_blocks_kernel<G>), dim3((uint32_t) blocks), dim3(256), 0, a.st, a.ix, a.qp, a.num,
                     a.steps, a.nwords, d_total);
  return hipGetLastError();
}


/* K in {1,2}; d in {32,64,128,192,256,448,960} */
#define KFMI_FOR_NB(X, K, LAY) \
  X(K, 1, LAY) X(K, 2, LAY) X(K, 4, LAY) X(K, 6, LAY) X(K, 8, LAY) X(K, 14, LAY) X(K, 30, LAY)


/* Locate: enough lanes to fill every CU (8 workgroups of 256 per CU), each
 * lane walking slot after slot (the cooperative walk: from its wave's share of
 * the slot queue). */
template <class G>
static hipError_t launch_locate(const SearchLaunch& a)
{
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
    cus = 256;
  uint64_t blocks = (a.total + 255) / 256;
  if constexpr (locate_coop_ok<G>()) {   /* MID lines: one round trip per step (KFMI_LOCATE_COOP=0: per-lane walk) */
    static const bool coop = [] {   /* KFMI_LOCATE_COOP, read once */
      const char* e = getenv("KFMI_LOCATE_COOP");
      return !e || atoi(e) != 0;
    }();
    if (coop) {
      /* 32 KB of LDS per workgroup: 5 fit a CU (4 measured the same within 2 %,
       * profiles/r02/locate_r2ba.jsonl: the walk is not short of lines in flight) */
      hipLaunchKernelGGL((locate_coop_kernel<G>), dim3(grid_blocks(blocks, (uint64_t) cus * 5)), dim3(256), 0, a.st, a.ix,
                         a.sa, a.sa_log2,
                         a.owner, a.total, a.pos, a.slot_ctr, a.slot_chunk);
      return hipGetLastError();
    }
  }
  hipLaunchKernelGGL((locate_kernel<G>), dim3(grid_blocks(blocks, (uint64_t) cus * 8)), dim3(256), 0, a.st, a.ix, a.sa,
                     a.sa_log2, a.owner, a.total, a.pos);
  return hipGetLastError();
}

template <class G>
static hipError_t launch_ftab(const SearchLaunch& a)
{
  const uint64_t blocks = (a.ftab_n + 255) / 256;
  hipLaunchKernelGGL((ftab_build_kernel<G>), dim3(grid_blocks(blocks, 1u << 20)), dim3(256), 0,
                     a.st, a.ix, a.ftab_steps, a.ftab_n, a.ftab_out);
  return hipGetLastError();
}

template <class G>
static hipError_t launch_rem_tab(const SearchLaunch& a)
{
  hipLaunchKernelGGL((rem_tab_kernel<G>), dim3(1), dim3(64), 0, a.st, a.ix, a.rem, a.ftab_out);
  return hipGetLastError();
}

template <class G>
static hipError_t launch_count_lines(const SearchLaunch& a, unsigned long long* d_out)
{
  const uint64_t blocks = (a.num + 255) / 256;
  hipLaunchKernelGGL((count_lines_kernel<G>), dim3((uint32_t) blocks), dim3(256), 0, a.st, a.ix, a.qp, a.num,
                     a.steps, a.nwords, d_out);
  return hipGetLastError();
}

template <class G>
static hipError_t launch_derive(const SearchLaunch& a)
{
  if constexpr (G::LAY == LAY_INTER && G::K <= 2) {
    hipLaunchKernelGGL((derive_codes_kernel<G>), dim3(grid_blocks((a.num + 255) / 256, 65536)), dim3(256), 0, a.st,
                       a.ix, a.num, a.derive_codes, a.derive_isa);
    return hipGetLastError();
  }
  return hipErrorInvalidValue;
}

template <class G>
static hipError_t launch_perm(const SearchLaunch& a)
{
  hipLaunchKernelGGL((lf_next_kernel<G>), dim3(grid_blocks((a.num + 255) / 256, 65536)), dim3(256), 0, a.st, a.ix,
                     a.num, a.perm_next, a.perm_bad);
  return hipGetLastError();
}

enum class Op { Task, Coop, Count, Locate, Ftab, RemTab, CountLines, Derive, PermCheck };

/* Defined here, instantiated once per (K, NB, LAY) in kfmi_inst_*.hip. */
template <int K, int NB, int LAY>
hipError_t dispatch_one(Op op, const SearchLaunch& a, unsigned long long* d_total)
{
  using G = Geo<K, NB, LAY>;
  switch (op) {
    case Op::Task: return launch_task<G>(a);
    case Op::Coop: return launch_coop<G>(a);
    case Op::Locate: return launch_locate<G>(a);
    case Op::Ftab: return launch_ftab<G>(a);
    case Op::RemTab: return launch_rem_tab<G>(a);
    case Op::CountLines: return launch_count_lines<G>(a, d_total);
    case Op::Derive: return launch_derive<G>(a);
    case Op::PermCheck: return launch_perm<G>(a);
    default: return launch_count<G>(a, d_total);
  }
}

#define KFMI_INSTANTIATE(KK, NBV, LAYV) \
  template hipError_t dispatch_one<KK, NBV, LAYV>(Op, const SearchLaunch&, unsigned long long*);
#define KFMI_EXTERN(KK, NBV, LAYV) \
  extern template hipError_t dispatch_one<KK, NBV, LAYV>(Op, const SearchLaunch&, unsigned long long*);

}  // namespace kfmi

#endif  // KFMI_KERNELS_H_
