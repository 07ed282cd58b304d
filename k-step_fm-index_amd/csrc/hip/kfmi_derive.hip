/*
 * kfmi_derive.hip -- a 2K-step index derived on the device from a K-step one
 * (layout tuning): the reference's K = 2 index file, without
 * its text, searched on the K = 4 grouped-counter layout (DESIGN.md 5d'),
 * its K = 1 files on K = 2.
 *
 * Row i of the K-step index (suffix p = SA[i]) holds the K-mer T[p-1-s],
 * s < K ('$' stored as A, genFMindex.c:505-509), and LF_K(i) is the row of
 * suffix p - K, whose K-mer is T[p-1-K-s]: so row i's 2K-mer is its own code
 * plus, above it, the code of row LF_K(i) (derive_codes_kernel,
 * kfmi_kernels.h, on the index's tag-101 layout: one row_code, one LF and one
 * row_code per row).  The exceptions are exact: the K rows D_s (s < K) whose
 * K-mer holds the '$' have no LF; their upper K bases are the text's tail
 * T[n-1-u], which row 0 (suffix n, an ordinary row) carries in its 2K-mer.  A
 * row whose LF lands on D_s is the row of suffix K + s, the new D_{K+s}.  From
 * the codes the builder's own steps (planes by ballot, per-code counts, scans,
 * C', build_from_codes in kfmi_build.hip) write the 2K-step entries, which
 * equal the index built from the text byte for byte (tests/test_derive.py).
 */
#include <vector>

#include "kfmi_runtime.h"

namespace kfmi {
int32_t build_from_codes(const uint8_t* d_codes, uint64_t n, uint32_t k, uint32_t d, const uint32_t* drow,
                         const uint32_t* dbase, int dev, bool host_image, kfmi_fmi_t** out);
}

namespace kfmi {

/* The derivation on device `dev` (current); the caller holds f's index lock
 * (shared is enough: f's own device copy is not touched). */
int32_t derive_index(kfmi_fmi_t* f, uint32_t k_out, int dev, bool host_image, kfmi_fmi_t** out)
{
  *out = nullptr;
  const uint32_t K = f->steps;
  if ((K != 1 && K != 2) || k_out != 2 * K) return KFMI_E_BAD_ARGUMENT;
  if (f->tag != KFMI_INDEX_VER_BASELINE && f->tag != KFMI_INDEX_VER_INTERLEAVE) return KFMI_E_BAD_ARGUMENT;
  const uint64_t rows = f->bwtsize, n = rows - 1;
  if (n < 2ull * k_out) return KFMI_E_BAD_ARGUMENT;   /* row 0's LF must not land on a '$' row */
  DevCtx* ctx = nullptr;
  int32_t err = ctx_for(dev, &ctx);
  if (err) return err;
  kfmi_dev_index* di = nullptr;
  err = upload_index(f, KFMI_BK_TASK, dev, ctx, &di);   /* the tag-101 layout, a copy of our own */
  if (err) return err;
  uint8_t* codes = nullptr;
  uint32_t* isa = nullptr;
  auto cleanup = [&]() {
    if (di) free_dev_index(di);
    di = nullptr;
    if (codes) (void) hipFree(codes);
    if (isa) (void) hipFree(isa);
    codes = nullptr;
    isa = nullptr;
  };
  /* the derivation composes LF_K with itself: only an index whose walks are
   * the text's (every row reaches a '$' row) has a 2K-step index to derive --
   * a 'ref'-mode index of a text with bytes other than A/C/G/T does not
   * (check_lf_walks) */
  err = check_lf_walks(di, ctx->st);
  if (!err && di->lf_perm.load() == 0) err = KFMI_E_BUILDING_FMI;
  if (err) {
    cleanup();
    return err;
  }
  if (hipMalloc((void**) &codes, rows) != hipSuccess || hipMalloc((void**) &isa, 16) != hipSuccess) {
    cleanup();
    return KFMI_E_DEVICE_ALLOC;
  }
  SearchLaunch a{};
  a.st = ctx->st;
  a.ix = idx_args(di);
  a.num = rows;
  a.derive_codes = codes;
  a.derive_isa = isa;
  uint32_t h_isa[4];
  uint8_t code0 = 0;
  if (hipMemsetAsync(isa, 0xFF, 16, ctx->st) != hipSuccess ||
      dispatch(Op::Derive, K, di->nb, di->layout, a) != hipSuccess ||
      hipMemcpyAsync(h_isa, isa, 16, hipMemcpyDeviceToHost, ctx->st) != hipSuccess ||
      hipMemcpyAsync(&code0, codes, 1, hipMemcpyDeviceToHost, ctx->st) != hipSuccess ||
      hipStreamSynchronize(ctx->st) != hipSuccess) {
    cleanup();
    return KFMI_E_KERNEL;
  }
  free_dev_index(di);   /* the tag-101 copy is no longer needed: free it before the build */
  di = nullptr;
  /* the new '$' rows: D_s for s < K are the K-step index's, D_{K+s} the rows
   * whose LF landed on D_s */
  uint32_t drow[4] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu}, dbase[4] = {0, 0, 0, 0};
  for (uint32_t s = 0; s < K; ++s) {
    drow[s] = f->dollarPositionBWT[s];
    drow[K + s] = h_isa[s];
  }
  for (uint32_t s = 0; s < k_out; ++s)
    if (drow[s] >= rows) {   /* not found: an inconsistent index (a 'ref'-mode walk that is not a permutation) */
      cleanup();
      return KFMI_E_BUILDING_FMI;
    }
  /* D_s, s < K: the K-mer as stored, then the text's tail above it -- base
   * t (K <= t < 2K) of suffix s's 2K-mer is T[n + s - t] = T[n - 1 - u] with
   * u = t - s - 1, which row 0's 2K-mer holds at bits 2u */
  for (uint32_t s = 0; s < K; ++s) {
    uint8_t low = 0;
    if (hipMemcpy(&low, codes + drow[s], 1, hipMemcpyDeviceToHost) != hipSuccess) {
      cleanup();
      return KFMI_E_KERNEL;
    }
    uint32_t code = low & ((1u << (2 * K)) - 1u);
    for (uint32_t t = K; t < 2 * K; ++t) code |= ((uint32_t) (code0 >> (2 * (t - s - 1))) & 3u) << (2 * t);
    const uint8_t c8 = (uint8_t) code;
    if (hipMemcpy(codes + drow[s], &c8, 1, hipMemcpyHostToDevice) != hipSuccess) {
      cleanup();
      return KFMI_E_KERNEL;
    }
  }
  for (uint32_t s = 0; s < k_out; ++s) {
    uint8_t c8 = 0;
    if (hipMemcpy(&c8, codes + drow[s], 1, hipMemcpyDeviceToHost) != hipSuccess) {
      cleanup();
      return KFMI_E_KERNEL;
    }
    dbase[s] = c8;
  }
  kfmi_fmi_t* g = nullptr;
  err = build_from_codes(codes, n, k_out, f->chunk, drow, dbase, dev, host_image, &g);
  cleanup();
  if (err) return err;
  *out = g;
  return KFMI_SUCCESS;
}

}  // namespace kfmi

using namespace kfmi;

extern "C" int32_t kfmi_derive_index_gpu(void* index, uint32_t k_out, int32_t want_host_image, void** out)
{
  kfmi_fmi_t* f = (kfmi_fmi_t*) index;
  if (!f || !out) return KFMI_E_BAD_ARGUMENT;
  *out = nullptr;
  if (kfmi_device_count() < 1) return KFMI_E_NO_DEVICE;
  DeviceGuard dg;
  std::shared_lock<RwLock> lk(index_lock(f));
  return derive_index(f, k_out, kfmi_current_device(), want_host_image != 0, (kfmi_fmi_t**) out);
}
