/*
 * copy_probe -- host <-> device copy rates for the transfer entry points
 * (dev tool, DESIGN.md 6a "Pageable transfers").
 *
 *   bin/copy_probe [GB=1.5] [threads=16]
 *
 * A pageable host buffer of GB gigabytes (malloc'd and touched, like
 * loadQueries' reads) and a device buffer of the same size; one JSON line per
 * form, the best of 3 runs:
 *   h2d_pageable_direct   hipMemcpy from the pageable buffer
 *   h2d_pinned_direct     hipMemcpy from a pinned (hipHostMalloc) buffer: the DMA ceiling
 *   host_memcpy_T         pageable -> pinned memcpy over T threads (the staging copy alone)
 *   h2d_staged_C_B_T      C-MB chunks through B pinned buffers, each filled by T threads
 *                         while the previous chunks' DMAs run (buffers allocated once,
 *                         outside the timing; the `alloc` rows add their hipHostMalloc)
 *   d2h_* the same for device -> host.
 */
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <thread>
#include <vector>

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

static double now()
{
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

/* memcpy over T threads, each a contiguous 4 KB-aligned part */
static void tcopy(void* dst, const void* src, uint64_t n, int T)
{
  if (T <= 1) {
    memcpy(dst, src, n);
    return;
  }
  const uint64_t part = ((n + T - 1) / T + 4095) & ~4095ull;
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t) {
    const uint64_t b = part * t;
    if (b >= n) break;
    const uint64_t len = std::min(part, n - b);
    th.emplace_back([=] { memcpy((uint8_t*) dst + b, (const uint8_t*) src + b, len); });
  }
  for (auto& x : th) x.join();
}

static void emit(const char* form, double s, uint64_t bytes)
{
  printf("{\"form\": \"%s\", \"ms\": %.2f, \"GB_s\": %.2f}\n", form, s * 1e3, bytes / s / 1e9);
  fflush(stdout);
}

static double best3(const std::function<void()>& f)
{
  double b = 1e30;
  for (int r = 0; r < 3; ++r) {
    const double t0 = now();
    f();
    b = std::min(b, now() - t0);
  }
  return b;
}

int main(int argc, char** argv)
{
  const double gb = argc > 1 ? atof(argv[1]) : 1.5;
  const int T = argc > 2 ? atoi(argv[2]) : 16;
  const uint64_t n = (uint64_t) (gb * 1e9) & ~4095ull;
  CHECK(hipSetDevice(0));
  uint8_t* page = (uint8_t*) malloc(n);
  uint8_t* back = (uint8_t*) malloc(n);
  if (!page || !back) return 1;
  for (uint64_t i = 0; i < n; i += 4096) page[i] = (uint8_t) i, back[i] = 0;
  memset(page, 'A', n);
  memset(back, 0, n);
  uint8_t *pin, *dev;
  CHECK(hipHostMalloc((void**) &pin, n, hipHostMallocDefault));
  CHECK(hipMalloc((void**) &dev, n));
  hipStream_t st;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  printf("{\"probe\": \"copy\", \"bytes\": %llu, \"threads\": %d}\n", (unsigned long long) n, T);

  emit("h2d_pageable_direct", best3([&] { CHECK(hipMemcpy(dev, page, n, hipMemcpyHostToDevice)); }), n);
  emit("h2d_pinned_direct", best3([&] {
         CHECK(hipMemcpyAsync(dev, pin, n, hipMemcpyHostToDevice, st));
         CHECK(hipStreamSynchronize(st));
       }), n);
  emit("d2h_pageable_direct", best3([&] { CHECK(hipMemcpy(back, dev, n, hipMemcpyDeviceToHost)); }), n);
  emit("d2h_pinned_direct", best3([&] {
         CHECK(hipMemcpyAsync(pin, dev, n, hipMemcpyDeviceToHost, st));
         CHECK(hipStreamSynchronize(st));
       }), n);
  for (int t : {1, 4, 8, 16, 32}) {
    if (t > 2 * T) break;
    char nm[64];
    snprintf(nm, sizeof nm, "host_memcpy_%d", t);
    emit(nm, best3([&] { tcopy(pin, page, n, t); }), n);
  }

  /* staged H2D / D2H through B pinned buffers of C MB */
  for (int cmb : {16, 32, 64}) {
    for (int B : {2, 3, 4}) {
      for (int t : {T / 2, T}) {
        if (t < 1) continue;
        const uint64_t C = (uint64_t) cmb << 20;
        std::vector<uint8_t*> buf(B);
        std::vector<hipEvent_t> ev(B);
        for (int b = 0; b < B; ++b) {
          CHECK(hipHostMalloc((void**) &buf[b], C, hipHostMallocDefault));
          CHECK(hipEventCreateWithFlags(&ev[b], hipEventDisableTiming));
        }
        auto h2d = [&] {
          uint64_t i = 0;
          for (uint64_t off = 0; off < n; off += C, ++i) {
            const int b = (int) (i % B);
            if (i >= (uint64_t) B) CHECK(hipEventSynchronize(ev[b]));
            const uint64_t len = std::min(C, n - off);
            tcopy(buf[b], page + off, len, t);
            CHECK(hipMemcpyAsync(dev + off, buf[b], len, hipMemcpyHostToDevice, st));
            CHECK(hipEventRecord(ev[b], st));
          }
          CHECK(hipStreamSynchronize(st));
        };
        /* D2H: DMA chunk i into buffer i % B, copy chunk i - (B-1) out while later DMAs run */
        auto d2h = [&] {
          const uint64_t nch = (n + C - 1) / C;
          for (uint64_t i = 0; i < nch + B - 1; ++i) {
            if (i < nch) {
              const int b = (int) (i % B);
              const uint64_t off = i * C, len = std::min(C, n - off);
              CHECK(hipMemcpyAsync(buf[b], dev + off, len, hipMemcpyDeviceToHost, st));
              CHECK(hipEventRecord(ev[b], st));
            }
            if (i + 1 >= (uint64_t) B) {
              const uint64_t j = i + 1 - B;
              if (j < nch) {
                const int b = (int) (j % B);
                CHECK(hipEventSynchronize(ev[b]));
                const uint64_t off = j * C, len = std::min(C, n - off);
                tcopy(back + off, buf[b], len, t);
              }
            }
          }
        };
        char nm[64];
        snprintf(nm, sizeof nm, "h2d_staged_%d_%d_%d", cmb, B, t);
        emit(nm, best3(h2d), n);
        snprintf(nm, sizeof nm, "d2h_staged_%d_%d_%d", cmb, B, t);
        emit(nm, best3(d2h), n);
        for (int b = 0; b < B; ++b) {
          CHECK(hipHostFree(buf[b]));
          CHECK(hipEventDestroy(ev[b]));
        }
      }
    }
  }
  /* the cost of pinning staging buffers per call */
  {
    const uint64_t C = 64ull << 20;
    emit("alloc_2x64MB_pinned", best3([&] {
           void *a, *b;
           CHECK(hipHostMalloc(&a, C, hipHostMallocDefault));
           CHECK(hipHostMalloc(&b, C, hipHostMallocDefault));
           CHECK(hipHostFree(a));
           CHECK(hipHostFree(b));
         }), 2 * C);
    emit("host_register_all", best3([&] {
           CHECK(hipHostRegister(page, n, hipHostRegisterDefault));
           CHECK(hipHostUnregister(page));
         }), n);
  }
  /* results check: the last staged D2H brought the device copy of `page` back */
  printf("{\"check\": %s}\n", memcmp(page, back, n) == 0 ? "true" : "false");
  CHECK(hipFree(dev));
  CHECK(hipHostFree(pin));
  free(page);
  free(back);
  return 0;
}
