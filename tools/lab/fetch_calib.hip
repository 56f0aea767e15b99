// fetch_calib.hip — lab probe (not product code): what rocprofv3's
// FETCH_SIZE / WRITE_SIZE report for the access shapes this repo's kernels
// use, against byte counts known by construction.  MI355X_MICROARCH.md
// calibrates only the 16-byte-per-lane streaming read (FETCH_SIZE = half the
// bytes) and 16-byte streaming stores (exact); "other access widths are
// uncalibrated".  Every table here is 1 GiB (4x the Infinity Cache), every
// gather index is a fixed random permutation, so each probe touches every
// byte it counts exactly once per launch.
//   hipcc --offload-arch=gfx950 -O3 -o tools/lab/bin/fetch_calib tools/lab/fetch_calib.hip
//   rocprofv3 --pmc FETCH_SIZE --output-format csv -d OUT -o run -- tools/lab/bin/fetch_calib
// Kernels (one launch each per repetition; bytes per launch printed):
//   p_stream16    16 B per lane, contiguous                     1 GiB read
//   p_stream8     8 B per lane, contiguous                      1 GiB read
//   p_stream1     1 B per lane, contiguous                      256 MiB read
//   p_row64       one 64-B row per 4 lanes (16 B each), random  16M rows = 1 GiB read
//   p_row128      one 128-B row per 8 lanes, random             8M rows = 1 GiB read
//   p_gather8     one 8-B word per lane, random 64-B segment    16M words (128 MiB useful)
//   p_store16     16 B per lane, contiguous                     1 GiB written
//   p_store40     one 40-B record per lane (struct copy), contiguous  640 MiB written
//   p_scatter8    one 8-B word per lane, random 64-B segment    16M words written
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <random>
#include <algorithm>

typedef uint32_t u32;
typedef uint64_t u64;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); return 1; } } while (0)

constexpr u64 kTable = 1ull << 30;  // bytes
constexpr u32 kBlock = 256;

__global__ __launch_bounds__(kBlock) void p_stream16(const uint4* __restrict__ a, u64 n, u32* out) {
  uint4 acc{0, 0, 0, 0};
  for (u64 i = u64(blockIdx.x) * kBlock + threadIdx.x; i < n; i += u64(gridDim.x) * kBlock) {
    const uint4 v = a[i];
    acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9E3779B9u) out[0] = 1;
}
__global__ __launch_bounds__(kBlock) void p_stream8(const u64* __restrict__ a, u64 n, u32* out) {
  u64 acc = 0;
  for (u64 i = u64(blockIdx.x) * kBlock + threadIdx.x; i < n; i += u64(gridDim.x) * kBlock) acc ^= a[i];
  if (acc == 0x9E3779B97F4A7C15ull) out[0] = 1;
}
__global__ __launch_bounds__(kBlock) void p_stream1(const uint8_t* __restrict__ a, u64 n, u32* out) {
  u32 acc = 0;
  for (u64 i = u64(blockIdx.x) * kBlock + threadIdx.x; i < n; i += u64(gridDim.x) * kBlock) acc += a[i];
  if (acc == 0x9E3779B9u) out[0] = 1;
}
// 4 lanes per row, lane q reads the row's q-th 16 bytes
__global__ __launch_bounds__(kBlock) void p_row64(const uint4* __restrict__ a, const u32* __restrict__ perm,
                                                  u64 rows, u32* out) {
  const u64 t = u64(blockIdx.x) * kBlock + threadIdx.x;
  const u64 r = t >> 2;
  if (r >= rows) return;
  const uint4 v = a[u64(perm[r]) * 4 + (t & 3)];
  if ((v.x ^ v.y ^ v.z ^ v.w) == 0x9E3779B9u) out[0] = 1;
}
// one lane per row, four 16-byte loads (the wire ingest's group-row read)
__global__ __launch_bounds__(kBlock) void p_row64_lane(const uint4* __restrict__ a,
                                                       const u32* __restrict__ perm, u64 rows, u32* out) {
  const u64 r = u64(blockIdx.x) * kBlock + threadIdx.x;
  if (r >= rows) return;
  const uint4* p = a + u64(perm[r]) * 4;
  const uint4 v0 = p[0], v1 = p[1], v2 = p[2], v3 = p[3];
  if ((v0.x ^ v1.y ^ v2.z ^ v3.w) == 0x9E3779B9u) out[0] = 1;
}
__global__ __launch_bounds__(kBlock) void p_row128(const uint4* __restrict__ a, const u32* __restrict__ perm,
                                                   u64 rows, u32* out) {
  const u64 t = u64(blockIdx.x) * kBlock + threadIdx.x;
  const u64 r = t >> 3;
  if (r >= rows) return;
  const uint4 v = a[u64(perm[r]) * 8 + (t & 7)];
  if ((v.x ^ v.y ^ v.z ^ v.w) == 0x9E3779B9u) out[0] = 1;
}
// one 8-byte word per lane, each in its own random 64-byte segment
__global__ __launch_bounds__(kBlock) void p_gather8(const u64* __restrict__ a, const u32* __restrict__ perm,
                                                    u64 n, u32* out) {
  const u64 t = u64(blockIdx.x) * kBlock + threadIdx.x;
  if (t >= n) return;
  if (a[u64(perm[t]) * 8] == 0x9E3779B97F4A7C15ull) out[0] = 1;
}
__global__ __launch_bounds__(kBlock) void p_store16(uint4* __restrict__ a, u64 n) {
  for (u64 i = u64(blockIdx.x) * kBlock + threadIdx.x; i < n; i += u64(gridDim.x) * kBlock)
    a[i] = uint4{u32(i), 1u, 2u, 3u};
}
struct Rec40 { u64 w[5]; };
__global__ __launch_bounds__(kBlock) void p_store40(Rec40* __restrict__ a, u64 n) {
  const u64 i = u64(blockIdx.x) * kBlock + threadIdx.x;
  if (i < n) a[i] = Rec40{{i, 1, 2, 3, 4}};
}
__global__ __launch_bounds__(kBlock) void p_scatter8(u64* __restrict__ a, const u32* __restrict__ perm, u64 n) {
  const u64 t = u64(blockIdx.x) * kBlock + threadIdx.x;
  if (t < n) a[u64(perm[t]) * 8] = t;
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 3;
  const u64 rows64 = kTable / 64, rows128 = kTable / 128;
  std::vector<u32> h(rows64);
  std::mt19937 rng(12345);
  for (u64 i = 0; i < rows64; ++i) h[i] = u32(i);
  std::shuffle(h.begin(), h.end(), rng);
  std::vector<u32> h2(rows128);
  for (u64 i = 0; i < rows128; ++i) h2[i] = u32(i);
  std::shuffle(h2.begin(), h2.end(), rng);
  char *tab, *tab2;
  u32 *perm, *perm2, *out;
  CK(hipMalloc(&tab, kTable));
  CK(hipMalloc(&tab2, kTable));
  CK(hipMalloc(&perm, rows64 * 4));
  CK(hipMalloc(&perm2, rows128 * 4));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(tab, 1, kTable));
  CK(hipMemset(tab2, 2, kTable));
  CK(hipMemcpy(perm, h.data(), rows64 * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(perm2, h2.data(), rows128 * 4, hipMemcpyHostToDevice));
  const u32 grid = 256 * 8;
  auto gr = [](u64 threads) { return u32((threads + kBlock - 1) / kBlock); };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char* name, u64 bytes, auto launch) -> int {
    float best = 1e30f;
    for (int r = 0; r < reps; ++r) {
      // evict: stream the other table between launches (writes, so nothing of it is re-read)
      hipLaunchKernelGGL(p_store16, dim3(grid), dim3(kBlock), 0, 0, reinterpret_cast<uint4*>(tab2),
                         kTable / 16);
      CK(hipEventRecord(e0));
      launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    printf("%-14s bytes %12llu  best %8.1f us  %6.2f TB/s\n", name, (unsigned long long)bytes,
           best * 1e3, bytes / (best * 1e-3) / 1e12);
    return 0;
  };
  run("p_stream16", kTable, [&] {
    hipLaunchKernelGGL(p_stream16, dim3(grid), dim3(kBlock), 0, 0, reinterpret_cast<const uint4*>(tab),
                       kTable / 16, out);
  });
  run("p_stream8", kTable, [&] {
    hipLaunchKernelGGL(p_stream8, dim3(grid), dim3(kBlock), 0, 0, reinterpret_cast<const u64*>(tab),
                       kTable / 8, out);
  });
  run("p_stream1", kTable / 4, [&] {
    hipLaunchKernelGGL(p_stream1, dim3(grid), dim3(kBlock), 0, 0, reinterpret_cast<const uint8_t*>(tab),
                       kTable / 4, out);
  });
  run("p_row64", kTable, [&] {
    hipLaunchKernelGGL(p_row64, dim3(gr(rows64 * 4)), dim3(kBlock), 0, 0,
                       reinterpret_cast<const uint4*>(tab), perm, rows64, out);
  });
  run("p_row64_lane", kTable, [&] {
    hipLaunchKernelGGL(p_row64_lane, dim3(gr(rows64)), dim3(kBlock), 0, 0,
                       reinterpret_cast<const uint4*>(tab), perm, rows64, out);
  });
  run("p_row128", kTable, [&] {
    hipLaunchKernelGGL(p_row128, dim3(gr(rows128 * 8)), dim3(kBlock), 0, 0,
                       reinterpret_cast<const uint4*>(tab), perm2, rows128, out);
  });
  run("p_gather8", rows64 * 8, [&] {
    hipLaunchKernelGGL(p_gather8, dim3(gr(rows64)), dim3(kBlock), 0, 0, reinterpret_cast<const u64*>(tab),
                       perm, rows64, out);
  });
  run("p_store16", kTable, [&] {
    hipLaunchKernelGGL(p_store16, dim3(grid), dim3(kBlock), 0, 0, reinterpret_cast<uint4*>(tab),
                       kTable / 16);
  });
  run("p_store40", 40ull * (kTable / 64), [&] {
    hipLaunchKernelGGL(p_store40, dim3(gr(kTable / 64)), dim3(kBlock), 0, 0, reinterpret_cast<Rec40*>(tab),
                       kTable / 64);
  });
  run("p_scatter8", rows64 * 8, [&] {
    hipLaunchKernelGGL(p_scatter8, dim3(gr(rows64)), dim3(kBlock), 0, 0, reinterpret_cast<u64*>(tab), perm,
                       rows64);
  });
  CK(hipDeviceSynchronize());
  return 0;
}
