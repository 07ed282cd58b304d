/*
 * kfmi_device.h -- device-side geometry and LF-mapping math for gfx950.
 *
 * One LF step of one interval end X with K-mer code c (the reference's
 * searchIndexCPU inner loop, fmIndexCPUBaseline.c:205-286):
 *   b = X / d, o = X % d
 *   X' = cnt_b[c] + popc( first-o-rows-mask & AND_{s<K} sel(plane_{s,0}, c_s.bit0) & sel(plane_{s,1}, c_s.bit1) )
 *        - #{s : D_s/d == b, c == dollarBase_s, X > D_s}
 * Two-sided form (AltCounters, fmIndexCPUBaseline-AltCounters.c:218-303): when
 * the counter sampled at the END of block b is used ("backward", e = 1),
 *   X' = cnt_{b+1}[c] - (popc(rows [o, d) of code c) - #{s : D_s/d == b, c == dollarBase_s, X <= D_s}).
 *
 * Device layouts (one per backend family; see DESIGN.md "Data layout in HBM"):
 *   LAY_INTER  : tag-101 entries as in the file, [planes(w,s,t) | cnt[NC]] u32
 *   LAY_AC     : tag-201 entries as in the file, [cnt_half[NC/2] | planes(w,s,t)];
 *                e = (b odd & c < NC/2) | (b even & c >= NC/2)
 *   LAY_MID    : one power-of-two line per PAIR of d-blocks (2d rows),
 *                [planes of block 2p | planes of block 2p+1 | cnt_{2p+1}[NC]]:
 *                every counter sits at the pair's midpoint, so an even block is
 *                searched backward (e = 1) and an odd block forward from the SAME
 *                line.  K=2, d=64: one 128-byte line per LF and nothing else --
 *                the AltCounters idea packed into one 128-B HBM request.
 *   LAY_MIDAC  : the LAY_MID lines with tag-201 (AltCounters) semantics.  The
 *                AltCounters searcher returns the true rank (= LAY_MID's
 *                result) in every block but the last real one (E-1) and the B5
 *                block E, where it counts back from the transform's sentinel
 *                counters (transformIndexAlternateCounters.c:420-431: '$' rows
 *                of block E-1 counted as their stored code, padding as A);
 *                blocks >= E-1 take that formula with the AC counters of
 *                entries E-1, E, E+1 (ix.ac_tail), everything else is LAY_MID.
 *   LAY_GRP    : K = 4 (256 counters per block): one power-of-two line per
 *                (d-block, group of 16 codes), [planes of block b | cnt_b[16g ..
 *                16g+15]], the planes repeated in the block's 16 lines.  K=4,
 *                d=64: 64 B of planes + 64 B of counters = one 128-B line per
 *                LF, 25 K-steps for a 100-bp read instead of 50 -- in 16 x
 *                the index memory (96 GB at 3 Gbase, which one MI355X holds).
 * Retired in round 6 (dominated on every measurement): the
 * packed layout (2: u16 counter deltas + superblock counters, 74 lines per
 * 100-bp read against MID128's 58) and AC128 (4: tag-201 semantics in one
 * 128-B line per block, 1,011 Mq/s against task-ac's 1,037-1,067 on the
 * reference's own tag-201 layout).  Their numbers stay unused.
 */
#ifndef KFMI_DEVICE_H_
#define KFMI_DEVICE_H_

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kfmi {

enum Layout : int { LAY_INTER = 0, LAY_AC = 1, LAY_MID = 3, LAY_MIDAC = 5, LAY_GRP = 6 };

__host__ __device__ constexpr int pow2ceil(int x) { int p = 1; while (p < x) p <<= 1; return p; }

template <int K_, int NB_, int LAY_>
struct Geo {
  static constexpr int K = K_;
  static constexpr int NB = NB_;                 // 32-row words per block
  static constexpr int LAY = LAY_;
  static constexpr int D = 32 * NB;              // rows per block (d)
  static constexpr int NC = 1 << (2 * K);        // counters (4^K)
  static constexpr int HALF = NC / 2;
  static constexpr int PW = 2 * K;               // planes per 32-row word
  static constexpr int BMW = PW * NB;            // bitmap words per block
  // u32 words per entry (per line for LAY_MID)
  static constexpr int NCG = NC < 16 ? NC : 16;          // counters per line (LAY_GRP)
  static constexpr int NGRP = NC / NCG;                   // lines per block (LAY_GRP)
  static constexpr int EW = LAY == LAY_INTER ? BMW + NC
                          : LAY == LAY_AC    ? HALF + BMW
                          : LAY == LAY_GRP    ? pow2ceil(BMW + NCG)
                          : pow2ceil(2 * BMW + NC);
  static constexpr int BOFF = LAY == LAY_AC ? HALF : 0;   // first bitmap word
  static constexpr int MIDCNT = 2 * BMW;                  // first mid counter (mid)
  static constexpr bool ACRULE = LAY == LAY_AC;          // AltCounters direction rule
  static constexpr int SPW = 32 / (2 * K);                // K-steps per packed query word
  static constexpr bool SMALL = BMW <= 16;                // whole bitmap fits in registers
  static constexpr bool TWO_SIDED = LAY == LAY_AC || LAY == LAY_MID || LAY == LAY_MIDAC;
  static constexpr bool MIDLINES = LAY == LAY_MID || LAY == LAY_MIDAC;   // pairs of blocks per line
  // the reference's own layouts (tag 101 / 201), register-resident blocks: a
  // block whose counter lies past the 128-B line of its planes is counted
  // forward from the previous block's counter when that entry lies in the
  // line (line_local_prev): one HBM line per LF where the layout allows it --
  // only where entry b-1 and block b's planes fit one 128-B line at all
  // (BOFF + EW + BMW words: K=2 d=64 and K=1 d<=128)
  static constexpr bool NEIGHBOR = (LAY == LAY_INTER || LAY == LAY_AC) && SMALL && BOFF + EW + BMW <= 32;
};

struct DollarArgs {
  uint32_t dpos[4];   // dollarPositionBWT[s], s < K <= 4
  uint32_t dbase[4];  // dollarBaseBWT[s]
  uint32_t dblk[4];   // dollarPositionBWT[s] / d (modposdollarBWT)
  uint32_t duniq;     // bit s: dpos[s] differs from every dpos[s'] with s' < s (a 'ref'-mode
                      // index can put two D_s on one row; its counters exclude that row once)
};

struct IdxArgs {
  const uint32_t* __restrict__ ent;   // entries / lines (layout per backend)
  uint32_t bwtsize;
  DollarArgs dl;
  // ftab (Bowtie-style jump start): [L, R) after the first ftab_steps K-steps,
  // indexed by the low 2*K*ftab_steps bits of the query's code stream; null = off
  const uint2* __restrict__ ftab;
  uint32_t ftab_steps, ftab_mask;
  // LAY_MIDAC: AltCounters counters of entries E-1, E (sentinel), E+1 (zero),
  // NC each, and E-1 = the first block that takes the AltCounters formula;
  // every AltCounters layout: row 3, the locate walk's correction of a step
  // backward from the sentinel (kfmi_search.hip ac_locate_fix)
  const uint32_t* __restrict__ ac_tail;
  uint32_t ac_tail_b0;
  // reads with m % K = rem != 0: [L, R) after their last rem bases (code of
  // bases m-1 .. m-rem at bits 0-1 ..), the start of their K-steps; null = rem 0
  const uint2* __restrict__ rtab;
  uint32_t rem;
  // task kernels: per-lane index gathers issued as exec-masked lane groups
  // (split_for, kfmi_search.hip: 4, 2 or 1 requested; launch_task picks the
  // fetch form).  A wave instruction whose 64 lanes hit 64 pages of a table
  // beyond the translation reach (~3.5 GB) stalls on translation; 16-32 pages
  // per instruction do not (profiles/r02/gather_mask_r2ag.jsonl)
  uint32_t split;
  // largest row an LF step may return (idx_args): the last row of the last
  // block every layout holds.  No result of a valid index comes near it (plain
  // results stay <= n+1 + d, AltCounters ones <= ac_clamp's cap); it keeps the
  // next step's loads inside the table when the counters or '$' rows of a
  // loaded file are corrupt (a wrapped or oversized counter).
  uint32_t lf_cap;
};

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef unsigned int v2u __attribute__((ext_vector_type(2)));

// 16/8/4-byte loads, optionally non-temporal (global_load ... nt): deep-step
// lines are touched once, so they should not evict the hot early-step lines.
template <bool NT>
__device__ __forceinline__ v4u ld4(const uint32_t* p)
{
  if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
  else return *reinterpret_cast<const v4u*>(p);
}
template <bool NT>
__device__ __forceinline__ v2u ld2(const uint32_t* p)
{
  if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const v2u*>(p));
  else return *reinterpret_cast<const v2u*>(p);
}
template <bool NT>
__device__ __forceinline__ uint32_t ld1(const uint32_t* p)
{
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}

// Bytes of alignment every block's bit planes are guaranteed to have (the
// layouts live in hipMalloc'd buffers, >= 256-byte aligned): the largest power
// of two dividing both 4*EW and 4*BOFF, at most 16.  Only the tag-201 layout
// at K = 1 falls short: its 4*(b*EW + HALF)-byte planes (EW = 2 + 2*NB words)
// are 8-byte aligned.
template <class G>
__host__ __device__ constexpr int plane_align()
{
  int a = 16;
  while (a > 4 && ((4 * G::EW) % a || (4 * G::BOFF) % a)) a >>= 1;
  return a;
}

// N consecutive index words at p as loads no wider than their alignment A
// (bytes).  Below 16, every load is fenced off by a compiler barrier: without
// it LLVM (load/store vectorizer, SILoadStoreOptimizer; unaligned-access-mode
// is on for gfx950) merges adjacent 8-byte loads into one 16-byte
// global_load_dwordx4 at an 8-mod-16 address, and that form, consumed under
// the partial s_waitcnt vmcnt(N > 0) the compiler schedules, is the round-5
// intermittent ftab table (one end one row off in ~1e-7 of the LF steps of
// lf_stream at K = 1, d = 64, tag 201).  The barrier emits no
// instruction; it only keeps the loads apart.
template <int A, int N, bool NT = false>
__device__ __forceinline__ void load_words(const uint32_t* __restrict__ p, uint32_t* __restrict__ out)
{
  if constexpr (A >= 16 && N % 4 == 0) {
#pragma unroll
    for (int i = 0; i < N / 4; ++i) {
      const v4u v = ld4<NT>(p + 4 * i);
      out[4 * i + 0] = v.x; out[4 * i + 1] = v.y; out[4 * i + 2] = v.z; out[4 * i + 3] = v.w;
    }
  } else if constexpr (A >= 8 && N % 2 == 0) {
#pragma unroll
    for (int i = 0; i < N / 2; ++i) {
      asm volatile("" ::: "memory");
      const v2u v = ld2<NT>(p + 2 * i);
      out[2 * i + 0] = v.x; out[2 * i + 1] = v.y;
    }
  } else {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      asm volatile("" ::: "memory");
      out[i] = ld1<NT>(p + i);
    }
  }
}

// base2index restated on a byte (genFMindex.c:71-84)
__device__ __forceinline__ uint32_t code_of(uint32_t x)
{
  uint32_t b1 = x & 4u, f2 = x & 2u;
  uint32_t b0 = b1 ? (f2 ^ 2u) : f2;
  return (b1 | b0) >> 1;
}

// Four ASCII bases (byte j = base j of the group) -> one byte of 2-bit codes in
// reverse order (base 3 at bits 0-1, base 0 at bits 6-7).  SWAR form of
// code_of on every byte: code = (bit2 << 1) | (bit1 ^ bit2).
__device__ __forceinline__ uint32_t group_codes_rev(uint32_t x)
{
  const uint32_t b1 = (x >> 2) & 0x01010101u;
  const uint32_t y = (b1 << 1) | (((x >> 1) & 0x01010101u) ^ b1);
  return ((y >> 24) & 0x03u) | ((y >> 14) & 0x0Cu) | ((y >> 4) & 0x30u) | ((y << 6) & 0xC0u);
}

// Shift the 2-bit code stream cw (cw[0] = lowest bits) left by `sh` bits
// (sh in {2,4,6,8}, wave-uniform) and insert `v` (sh bits) at the bottom.
template <int MAXW>
__device__ __forceinline__ void push_codes(uint32_t (&cw)[MAXW], uint32_t v, uint32_t sh)
{
#pragma unroll
  for (int k = MAXW - 1; k > 0; --k) cw[k] = __builtin_amdgcn_alignbit(cw[k], cw[k - 1], 32u - sh);
  cw[0] = (cw[0] << sh) | v;
}

// One ASCII row of m bases at base + off (any alignment; base 16-byte aligned,
// global or LDS) -> the reversed 2-bit stream the pack kernel writes: base
// m-1-r at bits 2r, so word w is packed word w of the query and K-step t sits
// at bits 2K*t (the order of fmIndexCPUBaseline.c:200-226).  Requires
// m <= 16*MAXW and 8 readable bytes past the row.
template <int MAXW>
__device__ __forceinline__ void row_codes(const uint8_t* __restrict__ base, uint64_t off, uint32_t m,
                                          uint32_t (&cw)[MAXW])
{
  const uint32_t* a = reinterpret_cast<const uint32_t*>(base + (off & ~3ull));
  const uint32_t sh = (uint32_t) (off & 3u);
  /* zeros written in place: as plain `cw[k] = 0` the compiler hoists MAXW
   * zero registers out of the staging loop and keeps them live beside the
   * working copy (MAXW = 16: 100 VGPRs, 5 waves/SIMD; this way 62, 8) */
#pragma unroll
  for (int k = 0; k < MAXW; ++k) asm volatile("v_mov_b32 %0, 0" : "=v"(cw[k]));
  const uint32_t ng = m >> 2, rem = m & 3u;
  uint32_t lo = a[0];
#pragma unroll 8
  for (uint32_t i = 0; i < ng; ++i) {
    const uint32_t hi = a[i + 1];
    push_codes<MAXW>(cw, group_codes_rev(__builtin_amdgcn_alignbyte(hi, lo, sh)), 8u);
    lo = hi;
  }
  if (rem) {
    const uint32_t x = __builtin_amdgcn_alignbyte(a[ng + 1], lo, sh);
    push_codes<MAXW>(cw, group_codes_rev(x) >> (2u * (4u - rem)), 2u * rem);
  }
}

// Code of the last `rem` bases of a row (base m-1 at bits 0-1): the remainder
// table's index for reads with m % K = rem.  p = the row's base m - rem.
__device__ __forceinline__ uint32_t rem_code(const uint8_t* __restrict__ p, uint32_t rem)
{
  uint32_t c = 0;
  for (uint32_t u = 0; u < rem; ++u) c |= code_of(p[rem - 1 - u]) << (2 * u);
  return c;
}

// K = 3: a K-step is 6 bits, so the pack kernel's words hold 5 steps (30 bits,
// SPW = 5) while the fused packers produce 16 bases per word; recut30 re-cuts
// the stream into 30-bit words with compile-time shifts (registers only).
template <int MAXW>
__host__ __device__ constexpr int k3_words() { return (MAXW * 32 + 29) / 30; }

template <int MAXW>
__device__ __forceinline__ void recut30(const uint32_t (&in)[MAXW], uint32_t (&out)[k3_words<MAXW>()])
{
#pragma unroll
  for (int j = 0; j < k3_words<MAXW>(); ++j) {
    const int bit = 30 * j, w = bit >> 5, sh = bit & 31;
    const uint32_t lo = w < MAXW ? in[w] : 0u;
    const uint32_t hi = w + 1 < MAXW ? in[w + 1] : 0u;
    out[j] = (sh ? ((lo >> sh) | (hi << (32 - sh))) : lo) & 0x3FFFFFFFu;
  }
}

// Fused query packing for a 256-thread block, one query per thread: each
// wave copies its rows HBM -> LDS with coalesced 16-byte loads, RPR rows per
// round, and the lanes owning those rows convert them from LDS (a lane reading
// its own row from HBM would touch a different line per lane).  LDS per wave:
// stage_slot_bytes(m).  Every thread of the block must call it.
__host__ __device__ constexpr uint32_t stage_rows(uint32_t m) { return m <= 128 ? 32u : 16u; }
__host__ __device__ constexpr uint32_t stage_slot_bytes(uint32_t m) { return (stage_rows(m) * m + 31u) & ~15u; }

template <int MAXW>
__device__ __forceinline__ void stage_query_codes(const uint8_t* __restrict__ ascii, uint64_t num, uint32_t m,
                                                  uint8_t* __restrict__ lds, uint32_t (&cw)[MAXW], uint32_t rem,
                                                  uint32_t& rc)
{
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint32_t rpr = stage_rows(m);
  uint8_t* wl = lds + wv * stage_slot_bytes(m);
  const uint64_t q0 = (uint64_t) blockIdx.x * 256 + wv * 64;
#pragma unroll 1
  for (uint32_t h = 0; h < 64u / rpr; ++h) {
    const uint64_t r0 = q0 + h * rpr;
    const uint64_t nr = r0 < num ? (num - r0 < rpr ? num - r0 : rpr) : 0;
    const uint32_t n16 = (uint32_t) ((nr * m + 15) / 16);           /* <= 15 bytes of slack read */
    const uint4* src = reinterpret_cast<const uint4*>(ascii + r0 * m);   /* r0*m % 16 == 0 */
    for (uint32_t i = lane; i < n16; i += 64) reinterpret_cast<uint4*>(wl)[i] = src[i];
    __syncthreads();
    if (lane / rpr == h) {   /* K-step stream of bases 0 .. m-rem-1; the rem last ones apart */
      row_codes<MAXW>(wl, (uint64_t) (lane % rpr) * m, m - rem, cw);
      rc = rem_code(wl + (uint64_t) (lane % rpr) * m + m - rem, rem);
    }
    __syncthreads();
  }
}

// first-`sh`-rows mask of one 32-row word, MSB = first row; sh clamped to [0,32]
__device__ __forceinline__ uint32_t row_mask(int sh)
{
  sh = sh < 0 ? 0 : (sh > 32 ? 32 : sh);
  return (uint32_t) ((0xFFFFFFFF00000000ull) >> sh);
}

// XOR masks selecting the planes of code c: plane p (= 2s+t) is used as is when
// bit p of c is set, inverted otherwise (fmIndexCPUBaseline.c:239-247).
template <int K>
__device__ __forceinline__ void plane_xor(uint32_t c, uint32_t (&sx)[2 * K])
{
#pragma unroll
  for (int p = 0; p < 2 * K; ++p) sx[p] = ((c >> p) & 1u) ? 0u : 0xFFFFFFFFu;
}

template <int K>
__device__ __forceinline__ uint32_t select_rows(const uint32_t* pl, const uint32_t (&sx)[2 * K])
{
  uint32_t v = ~0u;
#pragma unroll
  for (int p = 0; p < 2 * K; ++p) v &= pl[p] ^ sx[p];
  return v;
}

// Number of $ rows to discount (fmIndexCPUBaseline.c:252-256; AC :254-263).
template <int K, bool TWO>
__device__ __forceinline__ int dollar_fix(const DollarArgs& dl, uint32_t b, uint32_t c, uint32_t X, bool e)
{
  int corr = 0;
#pragma unroll
  for (int s = 0; s < K; ++s) {
    bool hit = (dl.dblk[s] == b) && (dl.dbase[s] == c);
    bool cond = (TWO && e) ? (X <= dl.dpos[s]) : (X > dl.dpos[s]);
    corr += (hit && cond) ? 1 : 0;
  }
  return corr;
}

// Direction and planes/counter addresses of block b for code c.
template <class G>
struct Where {
  const uint32_t* planes;
  const uint32_t* cnt;      // counter word
  bool e;                   // backward (two-sided layouts)
  bool prev = false;        // NEIGHBOR: counted forward from block b-1 (cnt is cnt_{b-1}[c])
  const uint32_t* pplanes = nullptr;   // NEIGHBOR, prev: the planes of block b-1
};

// Reference layouts (tag 101 INTER: [planes | cnt[NC]]; tag 201 AC:
// [cnt_half | planes]) in HBM as stored, 128-B lines.  When the counter the
// reference reads for (b, c) sits in another line than block b's planes --
// INTER, K=2, d=64: blocks b % 4 == 1 (entry [96, 192) of a line pair) and
// b % 4 == 2 with c >= 8; AC: odd blocks with c < NC/2, whose counter is entry
// b+1's -- but the whole previous entry b-1 lies in the planes' line (INTER
// b % 4 == 1; AC every odd b), the step is taken forward from cnt_{b-1}[c]:
//   X' = cnt_{b-1}[c] + popc(rows [start(b-1), X) of code c) - #{s : D_s in
//        blocks b-1, b, dollarBase_s == c, X > D_s}
// -- the same integer, since the reference builder derives every counter from
// the planes it stores (cnt_b = cnt_{b-1} + rows of block b-1 with code c,
// '$' rows excluded), so counts are consistent block to block.  The AC
// semantics differ from this only where the tfmiAC sentinel's counters are
// read (blocks >= E-1, ix.ac_tail_b0), which keep the reference's step.
// Which path a step takes changes no result, only the lines it touches:
// INTER 1.375 -> 1.125 lines per LF, AC 1.25 -> 1.
template <class G>
__device__ __forceinline__ void line_local_prev(const IdxArgs& ix, uint32_t b, uint32_t c, Where<G>& w)
{
  if constexpr (G::NEIGHBOR) {
    if (b == 0) return;
    const uint64_t pb = 4ull * ((uint64_t) b * G::EW + G::BOFF);   /* bytes: planes of block b */
    const uint64_t line = pb >> 7;
    if (((uint64_t) (w.cnt - ix.ent) * 4ull) >> 7 == line) return;  /* the reference's counter is in the line */
    if constexpr (G::LAY == LAY_AC) {
      if (!w.e || b >= ix.ac_tail_b0) return;   /* forward already, or the sentinel's counters */
    }
    const uint32_t cw = G::LAY == LAY_AC ? (c & (G::HALF - 1)) : (uint32_t) G::BMW + c;
    const uint64_t e0 = (uint64_t) (b - 1) * G::EW;
    if ((4ull * (e0 + G::BOFF)) >> 7 != line || (4ull * (e0 + G::BOFF + G::BMW) - 1) >> 7 != line ||
        (4ull * (e0 + cw)) >> 7 != line)
      return;
    w.prev = true;
    w.e = false;
    w.pplanes = ix.ent + e0 + G::BOFF;
    w.cnt = ix.ent + e0 + cw;
  }
}

template <class G>
__device__ __forceinline__ Where<G> locate(const IdxArgs& ix, uint32_t b, uint32_t c)
{
  Where<G> w;
  if constexpr (G::LAY == LAY_INTER) {
    const uint32_t* ent = ix.ent + (uint64_t) b * G::EW;
    w.planes = ent;
    w.cnt = ent + G::BMW + c;
    w.e = false;
  } else if constexpr (G::LAY == LAY_AC) {
    const uint32_t* ent = ix.ent + (uint64_t) b * G::EW;
    w.e = ((b & 1u) != 0) == (c < (uint32_t) G::HALF);
    w.planes = ent + G::BOFF;
    w.cnt = ix.ent + (uint64_t) (b + (w.e ? 1u : 0u)) * G::EW + (c & (G::HALF - 1));
  } else if constexpr (G::LAY == LAY_GRP) {
    const uint32_t* line = ix.ent + ((uint64_t) b * G::NGRP + c / G::NCG) * G::EW;
    w.planes = line;
    w.cnt = line + G::BMW + c % G::NCG;
    w.e = false;
  } else {   // LAY_MID, LAY_MIDAC
    const uint32_t* line = ix.ent + (uint64_t) (b >> 1) * G::EW;
    w.e = (b & 1u) == 0;                          // even block: backward from the midpoint
    w.planes = line + (b & 1u) * G::BMW;
    w.cnt = line + G::MIDCNT + c;
  }
  return w;
}

template <class G, bool NT = false>
__device__ __forceinline__ uint32_t load_counter(const IdxArgs& ix, const Where<G>& w, uint32_t b, uint32_t c)
{
  (void) ix; (void) b; (void) c;
  return ld1<NT>(w.cnt);
}

// AltCounters semantics past the last real block: the tfmiAC file ends with a
// sentinel entry S = ceil((n+1)/d) whose rows read as code 0, so on a text
// that ends in a run of A a step's result drifts past n+1 -- by up to K rows a
// step (a homopolymer of A walks R = n+1, n+3, ... at K=2) -- and stays
// defined while the step reads inside the file: block S counted forward, or
// any block below S.  Results reach (S+1)*d + K at most there.  Past that the
// reference reads past its own file (also B5) and its result is undefined; a
// wrapped value would send the next load out of the table.  Every
// AltCounters-semantics step is therefore capped at (S+2)*d - 1, which keeps
// every defined result and keeps the block index at most S+1, whose planes
// and counters every layout holds as zero padding (LAY_AC: entries S+1, S+2;
// LAY_MIDAC: the MID padding line and ac_tail row 2).
template <class G>
__device__ __forceinline__ uint32_t ac_clamp(const IdxArgs& ix, uint32_t v)
{
  const uint32_t cap = ((ix.bwtsize + (uint32_t) G::D - 1u) / (uint32_t) G::D + 2u) * (uint32_t) G::D - 1u;
  return v > cap ? cap : v;
}

// '$' rows of block b with code c that share their row with an earlier D_s
// (DollarArgs::duniq; only a 'ref'-mode index built from a text with non-ACGT
// bytes has them).  The reference's rule discounts one per s, its builder's
// counters one per row, so a step taken backward from cnt_{b+1} -- as the
// AltCounters searcher takes them (-AltCounters.c:254-266) -- lands this many
// rows above the forward step from cnt_b (fmIndexCPUBaseline.c:252-256).
template <int K>
__device__ __forceinline__ uint32_t dollar_dup(const DollarArgs& dl, uint32_t b, uint32_t c)
{
  uint32_t n = 0;
#pragma unroll
  for (int s = 1; s < K; ++s) n += (dl.dblk[s] == b && dl.dbase[s] == c && !((dl.duniq >> s) & 1u)) ? 1u : 0u;
  return n;
}

// the AltCounters direction of (b, c): backward from entry b+1
template <class G>
__device__ __forceinline__ bool ac_rule_e(uint32_t b, uint32_t c)
{
  return ((b & 1u) != 0) == (c < (uint32_t) G::HALF);
}

template <class G>
__device__ __forceinline__ uint32_t finish(const IdxArgs& ix, uint32_t cnt, uint32_t pop, uint32_t b, uint32_t c,
                                          uint32_t X, bool e)
{
  const int corr = dollar_fix<G::K, G::TWO_SIDED>(ix.dl, b, c, X, e);
  const uint32_t bc = pop - (uint32_t) corr;
  if constexpr (G::ACRULE) return ac_clamp<G>(ix, e ? cnt - bc : cnt + bc);
  if constexpr (G::MIDLINES) {
    // the MID direction is the block parity, not the semantics' own: give
    // back the forward step (MID) or the AltCounters one (MIDAC) where a
    // duplicated '$' row makes them differ (dollar_dup, nearly always 0)
    uint32_t v = e ? cnt - bc : cnt + bc;
    if (G::K > 1 && ix.dl.duniq != (1u << G::K) - 1u) {
      const uint32_t dup = dollar_dup<G::K>(ix.dl, b, c);
      const bool want = G::LAY == LAY_MIDAC && ac_rule_e<G>(b, c);
      v = v - (e ? dup : 0u) + (want ? dup : 0u);
    }
    return min(v, ix.lf_cap);
  }
  if constexpr (G::TWO_SIDED) return min(e ? cnt - bc : cnt + bc, ix.lf_cap);
  return min(cnt + bc, ix.lf_cap);
}

// line_local_prev's step: cnt = cnt_{b-1}[c], pop = rows of code c in block b-1
// and in rows [start(b), X) of block b; '$' rows of both blocks below X excluded
template <class G>
__device__ __forceinline__ uint32_t finish_prev(const IdxArgs& ix, uint32_t cnt, uint32_t pop, uint32_t b,
                                               uint32_t c, uint32_t X)
{
  int corr = 0;
#pragma unroll
  for (int s = 0; s < G::K; ++s) {
    if (ix.dl.dbase[s] != c) continue;
    if (ix.dl.dblk[s] == b) corr += X > ix.dl.dpos[s] ? 1 : 0;   // block b: the reference's own rule, per s
    else if (ix.dl.dblk[s] + 1u == b) corr += (ix.dl.duniq >> s) & 1u;   // block b-1: each '$' row once, as
  }                                                                  // the builder's counters exclude it
  uint32_t v = cnt + pop - (uint32_t) corr;
  // the AltCounters searcher takes this step backward from entry b+1: a
  // duplicated '$' row of block b lands it dollar_dup rows higher
  if constexpr (G::ACRULE) {
    if (G::K > 1 && ac_rule_e<G>(b, c)) v += dollar_dup<G::K>(ix.dl, b, c);
    return ac_clamp<G>(ix, v);
  }
  return min(v, ix.lf_cap);
}

// LAY_MIDAC, block b >= E-1: the AltCounters searcher's step
// (fmIndexCPUBaseline-AltCounters.c:218-303) from what the MID step already
// has -- its popcount over the MID direction (pop_mid; forward for odd b,
// backward for even b) and the block's whole count of code c (pop_all), so
// the AC direction's count is one of pop_mid or pop_all - pop_mid -- plus the
// AC counter of entry b or b+1 (ix.ac_tail; a rare, cached load).
template <class G>
__device__ __forceinline__ uint32_t ac_tail_step(const IdxArgs& ix, uint32_t b, uint32_t c, uint32_t X,
                                                 uint32_t pop_mid, uint32_t pop_all)
{
  const bool e = ((b & 1u) != 0) == (c < (uint32_t) G::HALF);
  const bool e_mid = (b & 1u) == 0;
  const uint32_t pop = e == e_mid ? pop_mid : pop_all - pop_mid;
  uint32_t row = b + (e ? 1u : 0u) - ix.ac_tail_b0;   /* 0, 1, 2: entries E-1, E, E+1 */
  row = row > 2u ? 2u : row;
  const uint32_t cnt = ix.ac_tail[row * (uint32_t) G::NC + c];
  const int corr = dollar_fix<G::K, true>(ix.dl, b, c, X, e);
  const uint32_t bc = pop - (uint32_t) corr;
  return ac_clamp<G>(ix, e ? cnt - bc : cnt + bc);
}

// ---------------------------------------------------------------------------
// Register-resident block fetch for small blocks (BMW <= 16 words): all bit
// planes of block b plus the one counter that code c needs.  Loads are
// 16-byte (dwordx4) when the plane group allows it.
// ---------------------------------------------------------------------------
template <class G>
struct Blk {
  uint32_t bm[G::BMW];
  uint32_t bp[G::NEIGHBOR ? G::BMW : 1];   // NEIGHBOR, prev: planes of block b-1
  uint32_t cnt;
  uint32_t b;
  bool e;
  bool prev;
};

template <class G, bool NT = false>
__device__ __forceinline__ void load_planes(const uint32_t* __restrict__ p, uint32_t (&bm)[G::BMW])
{
  load_words<plane_align<G>(), G::BMW, NT>(p, bm);
}

template <class G, bool NT = false>
__device__ __forceinline__ void fetch_block(const IdxArgs& ix, uint32_t b, uint32_t c, Blk<G>& k)
{
  Where<G> w = locate<G>(ix, b, c);
  line_local_prev<G>(ix, b, c, w);
  k.b = b;
  k.e = w.e;
  k.prev = w.prev;
  load_planes<G, NT>(w.planes, k.bm);
  if constexpr (G::NEIGHBOR) {
    if (w.prev) load_planes<G, NT>(w.pplanes, k.bp);
  }
  k.cnt = load_counter<G, NT>(ix, w, b, c);
}

template <class G>
__device__ __forceinline__ uint32_t lf_from_block(const IdxArgs& ix, const Blk<G>& k, uint32_t X, uint32_t c,
                                                  const uint32_t (&sx)[2 * G::K])
{
  const int o = (int) (X - k.b * (uint32_t) G::D);
  uint32_t pop = 0;
#pragma unroll
  for (int w = 0; w < G::NB; ++w) {
    uint32_t m = row_mask(o - 32 * w);
    if constexpr (G::TWO_SIDED) m = k.e ? ~m : m;
    pop += __popc(m & select_rows<G::K>(&k.bm[w * G::PW], sx));
  }
  if constexpr (G::LAY == LAY_MIDAC) {
    if (k.b >= ix.ac_tail_b0) {   /* rare: the last real block and past it */
      uint32_t all = 0;
#pragma unroll
      for (int w = 0; w < G::NB; ++w) all += __popc(select_rows<G::K>(&k.bm[w * G::PW], sx));
      return ac_tail_step<G>(ix, k.b, c, X, pop, all);
    }
  }
  if constexpr (G::NEIGHBOR) {
    if (k.prev) {   /* forward from cnt_{b-1}: all of block b-1, then rows [start(b), X) of block b */
#pragma unroll
      for (int w = 0; w < G::NB; ++w) pop += __popc(select_rows<G::K>(&k.bp[w * G::PW], sx));
      return finish_prev<G>(ix, k.cnt, pop, k.b, c, X);
    }
  }
  return finish<G>(ix, k.cnt, pop, k.b, c, X, k.e);
}

// ---------------------------------------------------------------------------
// Streaming LF for large blocks (d >= 192 with K=2): the planes are loaded in
// chunks of up to 8 words, every load of a chunk issued before any of its
// popcounts so the chunk's lines are in flight together; all words are read
// (as the reference does) and masked.  Also the per-row step of the ftab,
// remainder-table, derivation, statistics and locate kernels.  Loads follow
// load_words' alignment rule (the round-5 ftab hazard).
// ---------------------------------------------------------------------------
template <class G>
__device__ __forceinline__ uint32_t lf_stream(const IdxArgs& ix, uint32_t X, uint32_t c,
                                              const uint32_t (&sx)[2 * G::K])
{
  const uint32_t b = X / (uint32_t) G::D;
  const int o = (int) (X - b * (uint32_t) G::D);
  const Where<G> wh = locate<G>(ix, b, c);
  const uint32_t cnt = load_counter<G>(ix, wh, b, c);
  const uint32_t* pl = wh.planes;
  constexpr int CH = G::NB < 8 ? G::NB : 8;
  uint32_t pop = 0, all = 0;
#pragma unroll
  for (int w0 = 0; w0 < G::NB; w0 += CH) {
    uint32_t v[CH][G::PW];
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int w = w0 + j;
      if (w >= G::NB) break;
      load_words<plane_align<G>(), G::PW>(pl + G::PW * w, v[j]);   /* never wider than the planes' alignment */
    }
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int w = w0 + j;
      if (w >= G::NB) break;
      uint32_t m = row_mask(o - 32 * w);
      if constexpr (G::TWO_SIDED) m = wh.e ? ~m : m;
      const uint32_t sel = select_rows<G::K>(v[j], sx);
      pop += __popc(m & sel);
      if constexpr (G::LAY == LAY_MIDAC) all += __popc(sel);
    }
  }
  if constexpr (G::LAY == LAY_MIDAC)
    if (b >= ix.ac_tail_b0) return ac_tail_step<G>(ix, b, c, X, pop, all);
  return finish<G>(ix, cnt, pop, b, c, X, wh.e);
}

}  // namespace kfmi

#endif  // KFMI_DEVICE_H_
