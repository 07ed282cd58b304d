/*
 * kfmi_coop.h -- wave64-cooperative backward search (the reference's
 * Coop-{1,2}Step and Coop-2Step-AltCounters, fmIndexGPU-Coop-2Step.cu:147-228,
 * re-designed for CDNA4 instead of translated):
 *
 *  - one lane owns one query (both interval ends); a wave serves 64 queries;
 *  - per K-step every lane posts its L request and, only when R lies in a
 *    different d-block, an R request.  The R requests are compacted with a
 *    64-bit ballot + mbcnt (prefix popcount) so a wave issues 64 + popc(ballot)
 *    requests instead of 128;
 *  - TPR lanes fetch one request's Occ block (bit planes + the one 16-byte
 *    counter chunk it needs) with `global_load_lds_dwordx4`, straight from HBM
 *    into LDS (no VGPR staging); the 64/TPR requests of one round land as one
 *    contiguous 1 KiB piece;
 *  - after one vmcnt(0) every lane computes its own LF from its LDS slots.
 *
 * Results are identical to task_kernel (same lf math), hence to the CPU oracle.
 */
#ifndef KFMI_COOP_H_
#define KFMI_COOP_H_

#include <type_traits>

#include "kfmi_device.h"

namespace kfmi {

// NEIGHBOR geometries (reference tag-101/201 layouts, kfmi_device.h
// line_local_prev): a request's DMA carries block b's bit planes and either
// the 16-byte chunk holding its counter word or, when the step is counted
// forward from entry b-1, block b-1's planes -- whose counter word (same
// 128-B line, merged in L2 with the DMA's request) the lane owning that
// interval end then loads itself.  No request needs a second line's chunk.

template <class G>
struct CoopCfg {
  static constexpr int BC = G::BMW / 4;                 // 16-byte bitmap chunks per block
  static constexpr bool NBR = G::NEIGHBOR;              // planes of b + counter chunk, or of b and b-1
  static constexpr int TPR = NBR ? pow2ceil(2 * BC) : pow2ceil(BC + 1);   // lanes per request
  static constexpr int RPR = 64 / TPR;                  // requests per round
  static constexpr int SLOT = TPR * 16;                 // LDS bytes per request slot
  static constexpr int MAXREQ = 128;                    // 64 L + up to 64 R
  static constexpr int MAXR = MAXREQ / RPR;             // staging rounds per K-step, at most
  // a request's descriptor b * NC + c, posted by its lane; the staging round
  // that serves it decodes the chunk addresses (round 3 also measured lanes
  // posting ready-made addresses instead: neutral, removed in round 4,
  // DESIGN.md 5 "Coop issue")
  using Desc = typename std::conditional<(G::NC > 16), uint64_t, uint32_t>::type;
  static constexpr int WAVE_LDS = MAXREQ * SLOT + MAXREQ * (int) sizeof(Desc);
  static constexpr int WPB0 = 65536 / WAVE_LDS;
  static constexpr int WPB = WPB0 < 1 ? 1 : (WPB0 > 4 ? 4 : WPB0);   // waves per block
  static constexpr bool OK = (G::BMW % 4 == 0) && (G::EW % 4 == 0) && (G::BOFF % 4 == 0) &&
                             (!G::ACRULE || G::HALF >= 4) && (!G::MIDLINES || G::NC >= 4) &&
                             TPR <= 64;
};

// byte address of chunk k of request (b, c)
template <class G>
__device__ __forceinline__ const uint8_t* coop_chunk_addr(const IdxArgs& ix, uint32_t b, uint32_t c, int k)
{
  using C = CoopCfg<G>;
  const uint8_t* base = reinterpret_cast<const uint8_t*>(ix.ent);
  const uint64_t eb = (uint64_t) b * (G::EW * 4);
  if constexpr (G::MIDLINES) {
    const uint64_t lb = (uint64_t) (b >> 1) * (G::EW * 4);
    if (k < C::BC) return base + lb + ((b & 1u) * G::BMW + 4 * k) * 4;
    return base + lb + (G::MIDCNT + (c & ~3u)) * 4;
  }
  if constexpr (G::LAY == LAY_GRP) {
    const uint64_t lb = ((uint64_t) b * G::NGRP + c / G::NCG) * (G::EW * 4);
    if (k < C::BC) return base + lb + 16 * k;
    return base + lb + (G::BMW + ((c % G::NCG) & ~3u)) * 4;
  }
  if (k < C::BC) return base + eb + (G::BOFF + 4 * k) * 4;
  if constexpr (G::LAY == LAY_INTER) {
    return base + eb + (G::BMW + (c & ~3u)) * 4;
  } else {   // LAY_AC
    const bool e = ((b & 1u) != 0) == (c < (uint32_t) G::HALF);
    return base + (uint64_t) (b + (e ? 1u : 0u)) * (G::EW * 4) + ((c & (G::HALF - 1)) & ~3u) * 4;
  }
}

template <class G>
__device__ __forceinline__ uint32_t coop_lf(const IdxArgs& ix, const uint8_t* slot, uint32_t b, uint32_t X,
                                            uint32_t c, const uint32_t (&sx)[2 * G::K])
{
  using C = CoopCfg<G>;
  const int o = (int) (X - b * (uint32_t) G::D);
  bool e = false;
  if constexpr (G::ACRULE) e = ((b & 1u) != 0) == (c < (uint32_t) G::HALF);
  if constexpr (G::MIDLINES) e = (b & 1u) == 0;
  uint32_t pop = 0, all = 0;
  if constexpr (G::PW <= 4) {
#pragma unroll
    for (int k = 0; k < C::BC; ++k) {
      const uint4 v = *reinterpret_cast<const uint4*>(slot + 16 * k);
      const uint32_t pl[4] = {v.x, v.y, v.z, v.w};
      // K=2: one 32-row word per chunk; K=1: two words per chunk
#pragma unroll
      for (int h = 0; h < 4 / G::PW; ++h) {
        const int w = k * (4 / G::PW) + h;
        uint32_t m = row_mask(o - 32 * w);
        if constexpr (G::TWO_SIDED) m = e ? ~m : m;
        const uint32_t sel = select_rows<G::K>(&pl[h * G::PW], sx);
        pop += __popc(m & sel);
        if constexpr (G::LAY == LAY_MIDAC) all += __popc(sel);
      }
    }
  } else {   // K > 2: the block's BMW plane words (a 32-row word may straddle chunks at K = 3)
    uint32_t pl[G::BMW];
#pragma unroll
    for (int k = 0; k < C::BC; ++k) {
      const uint4 v = *reinterpret_cast<const uint4*>(slot + 16 * k);
      pl[4 * k] = v.x; pl[4 * k + 1] = v.y; pl[4 * k + 2] = v.z; pl[4 * k + 3] = v.w;
    }
#pragma unroll
    for (int w = 0; w < G::NB; ++w) {
      uint32_t m = row_mask(o - 32 * w);
      if constexpr (G::TWO_SIDED) m = e ? ~m : m;
      pop += __popc(m & select_rows<G::K>(&pl[w * G::PW], sx));
    }
  }
  const uint32_t cnt = reinterpret_cast<const uint32_t*>(slot + 16 * C::BC)[c & 3u];
  if constexpr (G::LAY == LAY_MIDAC)
    if (b >= ix.ac_tail_b0) return ac_tail_step<G>(ix, b, c, X, pop, all);
  return finish<G>(ix, cnt, pop, b, c, X, e);
}

// NEIGHBOR geometries: the slot holds block b's planes (chunks 0 .. BC-1) and,
// when w.prev, block b-1's (chunks BC .. 2BC-1), else the counter's chunk
// (chunk BC); cnt is the word w.cnt names.
template <class G>
__device__ __forceinline__ uint32_t coop_lf_nbr(const IdxArgs& ix, const uint8_t* slot, uint32_t b, uint32_t X,
                                                uint32_t c, const uint32_t (&sx)[2 * G::K], uint32_t cnt, bool e,
                                                bool prev)
{
  using C = CoopCfg<G>;
  const int o = (int) (X - b * (uint32_t) G::D);
  uint32_t pl[G::BMW];
#pragma unroll
  for (int k = 0; k < C::BC; ++k) {
    const uint4 v = *reinterpret_cast<const uint4*>(slot + 16 * k);
    pl[4 * k] = v.x; pl[4 * k + 1] = v.y; pl[4 * k + 2] = v.z; pl[4 * k + 3] = v.w;
  }
  uint32_t pop = 0;
#pragma unroll
  for (int w = 0; w < G::NB; ++w) {
    uint32_t m = row_mask(o - 32 * w);
    if constexpr (G::TWO_SIDED) m = e ? ~m : m;
    pop += __popc(m & select_rows<G::K>(&pl[w * G::PW], sx));
  }
  if (prev) {
#pragma unroll
    for (int k = 0; k < C::BC; ++k) {
      const uint4 v = *reinterpret_cast<const uint4*>(slot + 16 * (C::BC + k));
      pl[4 * k] = v.x; pl[4 * k + 1] = v.y; pl[4 * k + 2] = v.z; pl[4 * k + 3] = v.w;
    }
#pragma unroll
    for (int w = 0; w < G::NB; ++w) pop += __popc(select_rows<G::K>(&pl[w * G::PW], sx));
    return finish_prev<G>(ix, cnt, pop, b, c, X);
  }
  return finish<G>(ix, cnt, pop, b, c, X, e);
}

// Rows per staging round of the fused coop kernel: a multiple of 16 (so every
// round's source stays 16-byte aligned) whose bytes fit the wave's LDS area;
// 0 = the rows do not fit (use the pack kernel).
template <class G>
__host__ __device__ constexpr uint32_t coop_stage_rows(uint32_t m)
{
  uint32_t r = 64;
  while (r >= 16 && r * m + 16 > (uint32_t) CoopCfg<G>::WAVE_LDS) r >>= 1;
  return r >= 16 ? r : 0u;
}

// MAXW == 0: codes from the pack kernel's words (qp).  MAXW > 0: fused packing
// -- before its loop each wave copies its 64 ASCII rows HBM -> its own LDS area
// (coalesced 16-B loads, rounds of coop_stage_rows rows) and every lane turns
// its row into MAXW registers of codes; lanes past the batch end take the
// all-A query (valid rows for their DMA requests, never stored).
template <class G, int MAXW>
__global__ __launch_bounds__(64 * CoopCfg<G>::WPB) void coop_kernel(IdxArgs ix, const uint32_t* __restrict__ qp,
                                                                    const uint8_t* __restrict__ ascii, uint32_t m,
                                                                    uint64_t num, uint32_t steps, uint32_t nwords,
                                                                    uint32_t* __restrict__ res)
{
  using C = CoopCfg<G>;
  constexpr int RW = MAXW > 0 ? MAXW : 1;                                   // 16 bases per word
  constexpr int CW = MAXW > 0 && G::K == 3 ? k3_words<RW>() : RW;           // SPW K-steps per word
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  uint8_t* wl = lds + wave * C::WAVE_LDS;
  using Desc = typename C::Desc;
  Desc* tab = reinterpret_cast<Desc*>(wl + C::MAXREQ * C::SLOT);
  const uint64_t q0 = ((uint64_t) blockIdx.x * C::WPB + wave) * 64;
  if (q0 >= num) return;                       // whole wave idle (wave-uniform)
  const uint64_t q = q0 + lane;
  const uint64_t qs = q < num ? q : num - 1;   // tail lanes replay a valid query, never stored
  const int k = lane % C::TPR;
  const int g = lane / C::TPR;
  uint32_t cw[CW];
  uint32_t rc = 0;
  if constexpr (MAXW > 0) {
    uint32_t raw[RW];
    const uint32_t rpr = coop_stage_rows<G>(m);
#pragma unroll 1
    for (uint32_t h = 0; h < 64u / rpr; ++h) {
      const uint64_t r0 = q0 + h * rpr;
      const uint64_t nr = r0 < num ? (num - r0 < rpr ? num - r0 : rpr) : 0;
      const uint32_t n16 = (uint32_t) ((nr * m + 15) / 16);
      const uint4* src = reinterpret_cast<const uint4*>(ascii + r0 * m);
      for (uint32_t i = lane; i < n16; i += 64) reinterpret_cast<uint4*>(wl)[i] = src[i];
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      if ((uint32_t) lane / rpr == h) {   // K-step stream of bases 0 .. m-rem-1; the last rem apart
        row_codes<MAXW>(wl, (uint64_t) (lane % rpr) * m, m - ix.rem, raw);
        rc = rem_code(wl + (uint64_t) (lane % rpr) * m + m - ix.rem, ix.rem);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if (q >= num) {
#pragma unroll
      for (int i = 0; i < RW; ++i) raw[i] = 0;
      rc = 0;
    }
    if constexpr (G::K == 3) recut30<RW>(raw, cw);
    else {
#pragma unroll
      for (int i = 0; i < CW; ++i) cw[i] = raw[i];
    }
  }
  uint32_t L = 0, R = ix.bwtsize;
  uint32_t skip = 0;
  if (ix.ftab && steps >= ix.ftab_steps) {   // wave-uniform: jump start from the ftab
    skip = ix.ftab_steps;
    uint32_t w0;
    if constexpr (MAXW > 0) w0 = cw[0];
    else w0 = qp[qs];
    const uint2 lr = ix.ftab[w0 & ix.ftab_mask];
    L = lr.x;
    R = lr.y;
  }
  if (ix.rem) {   // wave-uniform: m % K != 0, the last rem bases from the remainder table
    if constexpr (MAXW == 0) rc = qp[(uint64_t) nwords * num + qs];
    const uint2 lr = ix.rtab[rc];
    L = lr.x;
    R = lr.y;
  }

  for (uint32_t w = 0; w < nwords; ++w) {
    uint32_t word;
    if constexpr (MAXW > 0) {
      word = cw[0];
#pragma unroll
      for (int i = 0; i + 1 < CW; ++i) cw[i] = cw[i + 1];
    } else {
      word = qp[(uint64_t) w * num + qs];
    }
    const uint32_t left = steps - w * G::SPW;
#pragma unroll 1
    for (int j = 0; j < G::SPW; ++j) {
      if ((uint32_t) j >= left) break;
      if (w * G::SPW + j < skip) continue;   // steps covered by the ftab (wave-uniform)
      const uint32_t c = (word >> (2 * G::K * j)) & (uint32_t) (G::NC - 1);
      const uint32_t bl = L / (uint32_t) G::D, br = R / (uint32_t) G::D;
      const bool needR = br != bl;
      const uint64_t mask = __ballot(needR);
      const uint32_t nreq = 64u + (uint32_t) __popcll(mask);
      const uint32_t slotR = 64u + __builtin_amdgcn_mbcnt_hi((uint32_t) (mask >> 32),
                                                             __builtin_amdgcn_mbcnt_lo((uint32_t) mask, 0u));
      bool eL = false, eR = false, pL = false, pR = false;
      const uint32_t* acL = nullptr;
      const uint32_t* acR = nullptr;
      if constexpr (C::NBR) {   // each end's counter word, loaded by its own lane after the DMA
        Where<G> wL = locate<G>(ix, bl, c);
        Where<G> wR = locate<G>(ix, br, c);
        line_local_prev<G>(ix, bl, c, wL);
        line_local_prev<G>(ix, br, c, wR);
        eL = wL.e;
        pL = wL.prev;
        acL = wL.cnt;
        eR = wR.e;
        pR = wR.prev;
        acR = wR.cnt;
      }
      tab[lane] = (Desc) bl * (Desc) G::NC + c;
      if (needR) tab[slotR] = (Desc) br * (Desc) G::NC + c;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      uint32_t cwL = 0, cwR = 0;   /* NBR: the counter word of an end that steps from block b-1 */
      const uint32_t rounds = (nreq + C::RPR - 1) / C::RPR;
      for (uint32_t r = 0; r < rounds; ++r) {
        const uint32_t s = r * C::RPR + g;
        if constexpr (C::NBR) {
          if (s < nreq && k < 2 * C::BC) {
            const Desc desc = tab[s];
            const uint32_t b = (uint32_t) (desc / (Desc) G::NC), cc = (uint32_t) (desc % (Desc) G::NC);
            Where<G> w = locate<G>(ix, b, cc);
            line_local_prev<G>(ix, b, cc, w);
            const uint32_t* p = k < C::BC ? w.planes + 4 * k
                                : w.prev ? w.pplanes + 4 * (k - C::BC)
                                : k == C::BC ? reinterpret_cast<const uint32_t*>(reinterpret_cast<uintptr_t>(w.cnt) & ~(uintptr_t) 15)
                                : nullptr;
            if (p)
              __builtin_amdgcn_global_load_lds((const void*) p,
                                               (__attribute__((address_space(3))) void*) (wl + r * 1024), 16, 0, 0);
          }
        } else if (s < nreq && k <= C::BC) {
          const Desc desc = tab[s];
          const uint32_t b = (uint32_t) (desc / (Desc) G::NC), cc = (uint32_t) (desc % (Desc) G::NC);
          const uint8_t* src = coop_chunk_addr<G>(ix, b, cc, k);
          __builtin_amdgcn_global_load_lds((const void*) src,
                                           (__attribute__((address_space(3))) void*) (wl + r * 1024), 16, 0, 0);
        }
      }
      if constexpr (C::NBR) {
        /* the counter words of the ends counted forward from block b-1 (the
         * others came with the DMA), after the DMA (their lines are then
         * already requested), as two exec-masked 32-lane groups (32 pages per
         * instruction at most, as the task kernels' fetch_ends_x4), R only
         * where it has its own block, parts no lane of a group needs branched
         * over; one vmcnt(0) for all */
        const uint64_t mpl = __ballot(pL), mpr = __ballot(needR && pR);
        uint64_t sv, gm;
        asm volatile("s_mov_b64 %[sv], exec\n"
                     "s_bfm_b64 %[gm], 32, 0\n"
                     "s_and_b64 exec, %[sv], %[gm]\n"
                     "s_and_b64 exec, exec, %[ml]\n"
                     "s_cbranch_execz .Lcl0_%=\n"
                     "global_load_dword %[cl], %[al], off\n"
                     ".Lcl0_%=:\n"
                     "s_and_b64 exec, %[sv], %[gm]\n"
                     "s_and_b64 exec, exec, %[mr]\n"
                     "s_cbranch_execz .Lcc0_%=\n"
                     "global_load_dword %[cr], %[ar], off\n"
                     ".Lcc0_%=:\n"
                     "s_bfm_b64 %[gm], 32, 32\n"
                     "s_and_b64 exec, %[sv], %[gm]\n"
                     "s_and_b64 exec, exec, %[ml]\n"
                     "s_cbranch_execz .Lcl1_%=\n"
                     "global_load_dword %[cl], %[al], off\n"
                     ".Lcl1_%=:\n"
                     "s_and_b64 exec, %[sv], %[gm]\n"
                     "s_and_b64 exec, exec, %[mr]\n"
                     "s_cbranch_execz .Lcc1_%=\n"
                     "global_load_dword %[cr], %[ar], off\n"
                     ".Lcc1_%=:\n"
                     "s_mov_b64 exec, %[sv]\n"
                     "s_waitcnt vmcnt(0)\n"
                     : [cl] "=&v"(cwL), [cr] "=&v"(cwR), [sv] "=&s"(sv), [gm] "=&s"(gm)
                     : [al] "v"(acL), [ar] "v"(acR), [ml] "s"(mpl), [mr] "s"(mpr)
                     : "memory", "scc");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      uint32_t sx[2 * G::K];
      plane_xor<G::K>(c, sx);
      uint32_t nL, nR;
      if constexpr (C::NBR) {
        /* the counter word: loaded above where that end steps from block b-1,
         * else word c % 4 of the slot's counter chunk (entries are 16-B
         * aligned and the counter index is c, or c mod NC/2, past a multiple
         * of 4 words) */
        const uint8_t* sL = wl + lane * C::SLOT;
        const uint8_t* sR = wl + (needR ? slotR : (uint32_t) lane) * C::SLOT;
        const uint32_t cL = pL ? cwL : reinterpret_cast<const uint32_t*>(sL + 16 * C::BC)[c & 3u];
        const uint32_t cR = needR ? (pR ? cwR : reinterpret_cast<const uint32_t*>(sR + 16 * C::BC)[c & 3u]) : cL;
        nL = coop_lf_nbr<G>(ix, sL, bl, L, c, sx, cL, eL, pL);
        nR = coop_lf_nbr<G>(ix, sR, br, R, c, sx, cR, needR ? eR : eL, needR ? pR : pL);
      } else {
        nL = coop_lf<G>(ix, wl + lane * C::SLOT, bl, L, c, sx);
        nR = coop_lf<G>(ix, wl + (needR ? slotR : (uint32_t) lane) * C::SLOT, br, R, c, sx);
      }
      L = nL;
      R = nR;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  }
  if (q < num) *reinterpret_cast<uint2*>(res + 2 * q) = make_uint2(L, R);
}

template <class G>
hipError_t coop_launch(hipStream_t st, IdxArgs ix, const uint32_t* qp, const uint8_t* ascii, uint32_t m, int maxw,
                       uint64_t num, uint32_t steps, uint32_t nwords, uint32_t* res)
{
  using C = CoopCfg<G>;
  if constexpr (!C::OK) {
    return hipErrorInvalidValue;
  } else {
    const uint64_t waves = (num + 63) / 64;
    const uint64_t blocks = (waves + C::WPB - 1) / C::WPB;
    const size_t lds = (size_t) C::WPB * C::WAVE_LDS;
    if (maxw == 8)
      hipLaunchKernelGGL((coop_kernel<G, 8>), dim3((uint32_t) blocks), dim3(64 * C::WPB), lds, st, ix, qp, ascii, m,
                         num, steps, nwords, res);
    else if (maxw == 16)
      hipLaunchKernelGGL((coop_kernel<G, 16>), dim3((uint32_t) blocks), dim3(64 * C::WPB), lds, st, ix, qp, ascii, m,
                         num, steps, nwords, res);
    else
      hipLaunchKernelGGL((coop_kernel<G, 0>), dim3((uint32_t) blocks), dim3(64 * C::WPB), lds, st, ix, qp, ascii, m,
                         num, steps, nwords, res);
    return hipGetLastError();
  }
}

}  // namespace kfmi

#endif  // KFMI_COOP_H_
