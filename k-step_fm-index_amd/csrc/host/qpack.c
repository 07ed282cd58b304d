/*
 * qpack.c -- host-side query packing for the streamed search.
 *
 * The search consumes a read as the 2-bit codes of its bases taken from the
 * last base backwards (fmIndexCPUBaseline.c:200-226: step t uses bases
 * m-1-K*t-i, i < K, base m-1-K*t in the low bits).  For K = 1 and K = 2 alike
 * that is one little-endian bit string: the base at reversed index r (base
 * m-1-r) sits at bits 2r..2r+1.  Word w of a read holds bits 32w..32w+31, so a
 * read of m bases has ceil(m/16) words and the bits past 2m are zero -- the
 * words the device pack kernel (csrc/hip/kfmi_search.hip, pack_queries_kernel)
 * writes.  Output is word-major, word w of read q at out[w * ostride + q], the
 * layout the LF kernels read coalesced.
 *
 * Packing on the host sends 4 bytes per 16 bases over PCIe instead of 16, for
 * kfmi_search_stream (streamed search).  Code of a base:
 * base2index (genFMindex.c:71-84) = ((x >> 1) & 3) ^ ((x >> 2) & 1).
 */
#define _GNU_SOURCE
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <immintrin.h>
#include "../kfmi_internal.h"

static inline uint32_t code2(uint8_t x)
{
  return ((uint32_t) (x >> 1) & 3u) ^ ((uint32_t) (x >> 2) & 1u);
}

/* Bases with reversed index >= r0 (positions m-1-r0 down to 0) into words
 * starting at word r0/16 (r0 a multiple of 16). */
static void pack_tail(const uint8_t* row, uint32_t m, uint32_t r0, uint32_t* out, uint64_t ostride)
{
  for (uint32_t w = r0 / 16; 16 * w < m; ++w) {
    uint32_t word = 0;
    for (uint32_t j = 0; j < 16 && 16 * w + j < m; ++j) word |= code2(row[m - 1 - (16 * w + j)]) << (2 * j);
    out[(uint64_t) w * ostride] = word;
  }
}

/* Every packer: rows at a, row q at a + q * stride, its first m bases packed
 * (stride >= m: a read whose last stride - m bases go to the remainder table). */
static void pack_rows_scalar(const uint8_t* a, uint64_t n, uint32_t stride, uint32_t m, uint32_t* out,
                             uint64_t ostride)
{
  for (uint64_t q = 0; q < n; ++q) pack_tail(a + q * stride, m, 0, out + q, ostride);
}

/* 32 bases per iteration: load, reverse, codes, 4 codes per byte. */
__attribute__((target("avx2"))) static void pack_rows_avx2(const uint8_t* a, uint64_t n, uint32_t stride, uint32_t m,
                                                           uint32_t* out, uint64_t ostride)
{
  const __m256i rev = _mm256_setr_epi8(15, 14, 13, 12, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2, 1, 0,
                                       15, 14, 13, 12, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2, 1, 0);
  const __m256i m3 = _mm256_set1_epi8(3), m1 = _mm256_set1_epi8(1);
  const __m256i w14 = _mm256_set1_epi16(0x0401);   /* maddubs: c0 + 4 c1 */
  const __m256i w116 = _mm256_set1_epi32(0x00100001);   /* madd: p0 + 16 p1 */
  const __m256i gather = _mm256_setr_epi8(0, 4, 8, 12, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1,
                                          0, 4, 8, 12, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1);
  const uint32_t full = m / 32;   /* 32-base groups from the end */
  for (uint64_t q = 0; q < n; ++q) {
    const uint8_t* row = a + q * stride;
    uint32_t* o = out + q;
    for (uint32_t k = 0; k < full; ++k) {
      __m256i v = _mm256_loadu_si256((const __m256i*) (row + m - 32 * (k + 1)));
      v = _mm256_shuffle_epi8(v, rev);
      v = _mm256_permute2x128_si256(v, v, 1);   /* byte j = base m-1-32k-j */
      const __m256i c = _mm256_xor_si256(_mm256_and_si256(_mm256_srli_epi16(v, 1), m3),
                                         _mm256_and_si256(_mm256_srli_epi16(v, 2), m1));
      const __m256i p = _mm256_madd_epi16(_mm256_maddubs_epi16(c, w14), w116);   /* 8 bits per dword */
      const __m256i b = _mm256_shuffle_epi8(p, gather);
      o[(uint64_t) (2 * k) * ostride] = (uint32_t) _mm256_extract_epi32(b, 0);
      o[(uint64_t) (2 * k + 1) * ostride] = (uint32_t) _mm256_extract_epi32(b, 4);
    }
    if (32 * full < m) pack_tail(row, m, 32 * full, o, ostride);
  }
}

/* 64 bases per block (AVX-512 BW + VBMI + VL, e.g. Zen 4/5 hosts), every
 * block branch-free: block k holds reversed bases 64k .. 64k+63.  A full block
 * is one unaligned load + one vpermb (reverse); the last, partial block of
 * cnt = m mod 64 bases is a masked load of the row's first cnt bytes (masked
 * bytes never fault, so the last row of a buffer is safe) + a zero-masking
 * vpermb.  Codes, 4 per byte (maddubs, madd), vpmovdb -> 16 bytes = 4 words;
 * zero bytes code as 0, the padding the words need past 2m bits. */
__attribute__((target("avx512f,avx512bw,avx512vbmi,avx512vl"))) static void pack_rows_avx512(const uint8_t* a,
                                                                                            uint64_t n, uint32_t stride,
                                                                                            uint32_t m, uint32_t* out,
                                                                                            uint64_t ostride)
{
  uint8_t ridx[64], tidx[64];
  const uint32_t full = m / 64, cnt = m % 64;
  for (int j = 0; j < 64; ++j) {
    ridx[j] = (uint8_t) (63 - j);
    tidx[j] = (uint8_t) (j < (int) cnt ? cnt - 1 - j : 0);
  }
  const __m512i rev = _mm512_loadu_si512((const void*) ridx), trev = _mm512_loadu_si512((const void*) tidx);
  const __mmask64 tmask = cnt ? (~0ull >> (64 - cnt)) : 0;
  const __m512i m3 = _mm512_set1_epi8(3), m1 = _mm512_set1_epi8(1);
  const __m512i w14 = _mm512_set1_epi16(0x0401), w116 = _mm512_set1_epi32(0x00100001);
  const uint32_t tw = (cnt + 15) / 16;   /* words of the partial block */
  for (uint64_t q = 0; q < n; ++q) {
    const uint8_t* row = a + q * stride;
    uint32_t* o = out + q;
    for (uint32_t k = 0; k <= full; ++k) {
      __m512i v;
      if (k < full) v = _mm512_permutexvar_epi8(rev, _mm512_loadu_si512((const void*) (row + m - 64 * (k + 1))));
      else if (cnt) v = _mm512_maskz_permutexvar_epi8(tmask, trev, _mm512_maskz_loadu_epi8(tmask, row));
      else break;
      const __m512i c = _mm512_xor_si512(_mm512_and_si512(_mm512_srli_epi16(v, 1), m3),
                                         _mm512_and_si512(_mm512_srli_epi16(v, 2), m1));
      const __m512i p = _mm512_madd_epi16(_mm512_maddubs_epi16(c, w14), w116);   /* 8 bits per dword */
      const __m128i b = _mm512_cvtepi32_epi8(p);                                 /* 16 bytes = 4 words */
      uint32_t* ow = o + (uint64_t) (4 * k) * ostride;
      const uint32_t nw = k < full ? 4 : tw;
      ow[0] = (uint32_t) _mm_extract_epi32(b, 0);
      if (nw > 1) ow[ostride] = (uint32_t) _mm_extract_epi32(b, 1);
      if (nw > 2) ow[2 * ostride] = (uint32_t) _mm_extract_epi32(b, 2);
      if (nw > 3) ow[3 * ostride] = (uint32_t) _mm_extract_epi32(b, 3);
    }
  }
}

/* KFMI_QPACK_ISA=scalar|avx2|avx512 pins the path (tests); default: the widest the host has.
 * rem = m % K bases at the end of every read go to the remainder table (DESIGN.md
 * 5e): the K-step stream covers bases 0 .. m-rem-1 (ceil((m-rem)/16) words) and
 * word row ceil((m-rem)/16) holds each read's remainder code (base m-1 at bits
 * 0-1, base m-2 at 2-3, ...) -- the rows pack_queries_kernel writes. */
void kfmi_pack_rows_rem(const uint8_t* ascii, uint64_t n, uint32_t m, uint32_t rem, uint32_t* out, uint64_t ostride)
{
  static int isa = -1;   /* 0 scalar, 1 avx2, 2 avx512 */
  const char* e = getenv("KFMI_QPACK_ISA");
  int use;
  if (isa < 0) {
    isa = 0;
    if (__builtin_cpu_supports("avx2")) isa = 1;
    if (isa && __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
        __builtin_cpu_supports("avx512vbmi") && __builtin_cpu_supports("avx512vl"))
      isa = 2;
  }
  use = isa;
  if (e) {
    const int want = !strcmp(e, "scalar") ? 0 : !strcmp(e, "avx2") ? 1 : 2;
    use = want < isa ? want : isa;
  }
  const uint32_t mk = m - rem;
  if (use == 2) pack_rows_avx512(ascii, n, m, mk, out, ostride);
  else if (use == 1) pack_rows_avx2(ascii, n, m, mk, out, ostride);
  else pack_rows_scalar(ascii, n, m, mk, out, ostride);
  if (rem) {
    uint32_t* o = out + (uint64_t) ((mk + 15) / 16) * ostride;
    for (uint64_t q = 0; q < n; ++q) {
      const uint8_t* row = ascii + q * m;
      uint32_t c = 0;
      for (uint32_t u = 0; u < rem; ++u) c |= code2(row[m - 1 - u]) << (2 * u);
      o[q] = c;
    }
  }
}

void kfmi_pack_rows(const uint8_t* ascii, uint64_t n, uint32_t m, uint32_t* out, uint64_t ostride)
{
  kfmi_pack_rows_rem(ascii, n, m, 0, out, ostride);
}

int32_t kfmi_pack_queries(const char* ascii, uint64_t num, uint32_t size, uint32_t* words)
{
  if ((!ascii || !words) && num) return KFMI_E_BAD_ARGUMENT;
  if (size == 0) return KFMI_E_BAD_ARGUMENT;
  kfmi_pack_rows((const uint8_t*) ascii, num, size, words, num);
  return KFMI_SUCCESS;
}

int32_t kfmi_pack_queries_k(const char* ascii, uint64_t num, uint32_t size, uint32_t k, uint32_t* words)
{
  if ((!ascii || !words) && num) return KFMI_E_BAD_ARGUMENT;
  if (size == 0 || (k != 1 && k != 2 && k != 4)) return KFMI_E_BAD_ARGUMENT;
  kfmi_pack_rows_rem((const uint8_t*) ascii, num, size, size % k, words, num);
  return KFMI_SUCCESS;
}
