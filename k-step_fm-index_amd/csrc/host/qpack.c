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

static void pack_rows_scalar(const uint8_t* a, uint64_t n, uint32_t m, uint32_t* out, uint64_t ostride)
{
  for (uint64_t q = 0; q < n; ++q) pack_tail(a + q * m, m, 0, out + q, ostride);
}

/* 32 bases per iteration: load, reverse, codes, 4 codes per byte. */
__attribute__((target("avx2"))) static void pack_rows_avx2(const uint8_t* a, uint64_t n, uint32_t m, uint32_t* out,
                                                           uint64_t ostride)
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
    const uint8_t* row = a + q * m;
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

void kfmi_pack_rows(const uint8_t* ascii, uint64_t n, uint32_t m, uint32_t* out, uint64_t ostride)
{
  static int avx2 = -1;
  if (avx2 < 0) avx2 = __builtin_cpu_supports("avx2") ? 1 : 0;
  if (avx2) pack_rows_avx2(ascii, n, m, out, ostride);
  else pack_rows_scalar(ascii, n, m, out, ostride);
}

int32_t kfmi_pack_queries(const char* ascii, uint64_t num, uint32_t size, uint32_t* words)
{
  if ((!ascii || !words) && num) return KFMI_E_BAD_ARGUMENT;
  if (size == 0) return KFMI_E_BAD_ARGUMENT;
  kfmi_pack_rows((const uint8_t*) ascii, num, size, words, num);
  return KFMI_SUCCESS;
}
