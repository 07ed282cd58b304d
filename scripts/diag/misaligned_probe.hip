// Probe: 16-byte loads at 8-byte-aligned addresses (a 24-byte record stride,
// the layout of the K = 1, d = 64 AltCounters entries), many lanes of a wave
// sharing one address, some straddling a 128-B line -- the access shape of
// the ftab build that returned intermittent wrong entries.  Each lane loads
// its record's 16 bytes as two 8-byte halves (merged by the compiler into one
// dwordx4) and compares them with the known contents; mismatches counted.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void probe(const uint32_t* __restrict__ buf, uint32_t nrec, uint32_t share, uint32_t iters,
                      unsigned long long* __restrict__ bad, uint32_t salt)
{
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t errs = 0;
  for (uint32_t it = 0; it < iters; ++it) {
    uint32_t rec = ((gid / share) * 2654435761u + it * 40503u + salt) % nrec;   // lanes share records
    const uint32_t* p = buf + (uint64_t) rec * 6 + 2;                           // 24-B stride, +8 B
    const uint2 a = *reinterpret_cast<const uint2*>(p);
    const uint2 b = *reinterpret_cast<const uint2*>(p + 2);
    const uint32_t w = rec * 6 + 2;
    errs += (a.x != w * 2654435761u) + (a.y != (w + 1) * 2654435761u) + (b.x != (w + 2) * 2654435761u) +
            (b.y != (w + 3) * 2654435761u);
  }
  if (errs) atomicAdd(bad, (unsigned long long) errs);
}

int main(int argc, char** argv)
{
  const uint32_t nrec = argc > 1 ? atoi(argv[1]) : 46879;
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  std::vector<uint32_t> h((size_t) nrec * 6 + 8);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (uint32_t) i * 2654435761u;
  uint32_t* d = nullptr;
  unsigned long long* bad = nullptr;
  hipMalloc(&d, h.size() * 4);
  hipMalloc(&bad, 8);
  hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  for (uint32_t share : {1u, 4u, 16u, 64u}) {
    unsigned long long total = 0;
    for (int r = 0; r < reps; ++r) {
      hipMemset(bad, 0, 8);
      hipLaunchKernelGGL(probe, dim3(65536), dim3(256), 0, 0, d, nrec, share, 64, bad, (uint32_t) r * 7919u);
      unsigned long long b = 0;
      hipMemcpy(&b, bad, 8, hipMemcpyDeviceToHost);
      total += b;
    }
    printf("share %2u lanes per record: %llu wrong words in %llu loads of 16 B\n", share, total,
           (unsigned long long) reps * 65536ull * 256ull * 64ull);
  }
  hipFree(d);
  hipFree(bad);
  return 0;
}
