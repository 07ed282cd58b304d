// Standalone repro of the round-5 intermittent ftab table:
// the table of the K = 1, d = 64 AltCounters layout built by the old per-end
// step (lf_stream, "A") against the task kernels' step (fetch_block +
// lf_from_block, "B"), several builds each, entries compared.
//   ftab_repro <tag-201 image file> [builds] [fsteps]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "kfmi_device.h"

using namespace kfmi;
using G = Geo<1, 2, LAY_AC>;

__global__ __launch_bounds__(256) void build_a(IdxArgs ix, uint32_t fsteps, uint64_t n, uint2* __restrict__ out)
{
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

__global__ __launch_bounds__(256) void build_b(IdxArgs ix, uint32_t fsteps, uint64_t n, uint2* __restrict__ out)
{
  for (uint64_t v = (uint64_t) blockIdx.x * 256 + threadIdx.x; v < n; v += (uint64_t) gridDim.x * 256) {
    uint32_t L = 0, R = ix.bwtsize;
    for (uint32_t t = 0; t < fsteps; ++t) {
      const uint32_t c = (uint32_t) (v >> (2 * G::K * t)) & (uint32_t) (G::NC - 1);
      uint32_t sx[2 * G::K];
      plane_xor<G::K>(c, sx);
      Blk<G> kl, kr;
      fetch_block<G>(ix, L / (uint32_t) G::D, c, kl);
      fetch_block<G>(ix, R / (uint32_t) G::D, c, kr);
      L = lf_from_block<G>(ix, kl, L, c, sx);
      R = lf_from_block<G>(ix, kr, R, c, sx);
    }
    out[v] = make_uint2(L, R);
  }
}

int main(int argc, char** argv)
{
  if (argc < 2) { fprintf(stderr, "usage: %s image201 [builds] [fsteps]\n", argv[0]); return 2; }
  const int builds = argc > 2 ? atoi(argv[2]) : 8;
  const uint32_t fsteps = argc > 3 ? (uint32_t) atoi(argv[3]) : 12;
  FILE* fp = fopen(argv[1], "rb");
  if (!fp) return 3;
  std::vector<uint32_t> img;
  uint32_t w;
  while (fread(&w, 4, 1, fp) == 1) img.push_back(w);
  fclose(fp);
  const uint32_t tag = img[0], K = img[1], bwtsize = img[2], nentries = img[4], chunk = img[5];
  if (tag != 201 || K != 1 || chunk != 64) { fprintf(stderr, "want a K=1 d=64 tag-201 image\n"); return 4; }
  const uint32_t ew = G::EW;
  std::vector<uint32_t> ent(img.begin() + 8, img.begin() + 8 + (size_t) ew * nentries);
  ent.resize(ent.size() + 2 * ew, 0u);   // two zero padding entries, as the AC device layout
  uint32_t* d_ent = nullptr;
  hipMalloc(&d_ent, ent.size() * 4);
  hipMemcpy(d_ent, ent.data(), ent.size() * 4, hipMemcpyHostToDevice);
  IdxArgs ix{};
  ix.ent = d_ent;
  ix.bwtsize = bwtsize;
  for (int s = 0; s < 4; ++s) {
    ix.dl.dpos[s] = s < 1 ? img[6] : 0xFFFFFFFFu;
    ix.dl.dbase[s] = s < 1 ? img[7] : 0xFFFFFFFFu;
    ix.dl.dblk[s] = s < 1 ? img[6] / chunk : 0xFFFFFFFFu;
  }
  ix.dl.duniq = 1;
  ix.ac_tail_b0 = nentries >= 2 ? nentries - 2 : 0;
  ix.split = 1;
  const uint64_t n = 1ull << (2 * fsteps);
  const uint64_t blocks = (n + 255) / 256;
  const uint32_t grid = (uint32_t) (blocks < (1u << 20) ? blocks : (1u << 20));
  std::vector<uint2> ref(n), got(n);
  uint2* t = nullptr;
  hipMalloc(&t, n * 8);
  hipLaunchKernelGGL(build_b, dim3(grid), dim3(256), 0, 0, ix, fsteps, n, t);
  hipMemcpy(ref.data(), t, n * 8, hipMemcpyDeviceToHost);
  const bool fresh = argc > 4 && atoi(argv[4]) != 0;   // the library's sequence: fresh upload + table per build
  hipStream_t st = nullptr;
  hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  for (const char* which : {"B", "A"}) {
    for (int b = 0; b < builds; ++b) {
      if (fresh) {
        hipFree(t);
        hipFree(d_ent);
        std::vector<uint32_t> junk(n * 2, 0x5A5A5A5Au);   // something else lives at those addresses first
        uint32_t* other = nullptr;
        hipMalloc(&other, n * 8 + ent.size() * 4);
        hipMemcpy(other, junk.data(), n * 8, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(build_b, dim3(grid), dim3(256), 0, 0, ix, 2u, n / 4, reinterpret_cast<uint2*>(other));
        hipDeviceSynchronize();
        hipFree(other);
        hipMalloc(&d_ent, ent.size() * 4);
        hipMemcpyAsync(d_ent, ent.data(), ent.size() * 4, hipMemcpyHostToDevice, 0);
        hipStreamSynchronize(0);
        ix.ent = d_ent;
        hipMalloc(&t, n * 8);
      } else {
        hipMemset(t, 0xAB, n * 8);
      }
      if (which[0] == 'A') hipLaunchKernelGGL(build_a, dim3(grid), dim3(256), 0, st, ix, fsteps, n, t);
      else hipLaunchKernelGGL(build_b, dim3(grid), dim3(256), 0, st, ix, fsteps, n, t);
      hipStreamSynchronize(st);
      hipMemcpy(got.data(), t, n * 8, hipMemcpyDeviceToHost);
      uint64_t bad = 0, first = ~0ull;
      for (uint64_t v = 0; v < n; ++v)
        if (got[v].x != ref[v].x || got[v].y != ref[v].y) { if (!bad) first = v; ++bad; }
      printf("build %s #%d: %llu entries differ from B's first build", which, b, (unsigned long long) bad);
      if (bad) printf(" (first v=%llu: %u %u vs %u %u)", (unsigned long long) first, got[first].x, got[first].y,
                      ref[first].x, ref[first].y);
      printf("\n");
      fflush(stdout);
    }
  }
  return 0;
}
