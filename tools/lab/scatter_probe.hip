// scatter_probe.hip — lab probe (not product code): can the tracker step's
// two-level bucketing (K3 scatter to super-buckets + K4 split to chunks) be
// one pass?  One 64K-record tile per CU, an LDS table of 32768 chunk bases
// (128 KB), LDS atomic ranks, one scattered 16-byte store per record.
// Measures hist / scan / scatter times for 16M records over 16M groups in
// random order (the config-5 stream's shape).
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/scatter_probe tools/lab/scatter_probe.hip
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

constexpr u32 kChunkShift = 9;         // 512 groups per chunk
constexpr u32 kTiles = 256;
constexpr u32 kBlock = 1024;
constexpr u32 kSegs = 8;

__global__ __launch_bounds__(kBlock) void k_hist(const u32* __restrict__ grp, u64 M, u32 C, u32 T,
                                                 u32* __restrict__ H) {
  extern __shared__ u32 h[];
  for (u32 c = threadIdx.x; c < C; c += kBlock) h[c] = 0;
  __syncthreads();
  const u64 t0 = u64(blockIdx.x) * T;
  const u64 t1 = t0 + T < M ? t0 + T : M;
  for (u64 j = t0 + threadIdx.x * 4; j < t1; j += kBlock * 4) {
    const uint4 g = *reinterpret_cast<const uint4*>(grp + j);
    atomicAdd(&h[g.x >> kChunkShift], 1u);
    atomicAdd(&h[g.y >> kChunkShift], 1u);
    atomicAdd(&h[g.z >> kChunkShift], 1u);
    atomicAdd(&h[g.w >> kChunkShift], 1u);
  }
  __syncthreads();
  u32* row = H + u64(blockIdx.x) * C;
  for (u32 c = threadIdx.x; c < C; c += kBlock) row[c] = h[c];
}

// part[s][c] = sum over the tiles of segment s of H[t][c]
__global__ void k_scan_a(const u32* __restrict__ H, u32 C, u32* __restrict__ part) {
  const u32 c = blockIdx.x * blockDim.x + threadIdx.x;
  const u32 s = blockIdx.y;
  if (c >= C) return;
  const u32 per = kTiles / kSegs;
  u32 v[kTiles / kSegs];
#pragma unroll
  for (u32 i = 0; i < per; ++i) v[i] = H[u64(s * per + i) * C + c];
  u32 sum = 0;
#pragma unroll
  for (u32 i = 0; i < per; ++i) sum += v[i];
  part[u64(s) * C + c] = sum;
}

// one block: base[c] = exclusive scan of chunk totals; part[s][c] -> segment base
__global__ __launch_bounds__(1024) void k_scan_b(u32* __restrict__ part, u32 C, u32* __restrict__ base) {
  __shared__ u32 ws[1024];
  const u32 per = (C + 1023) / 1024;
  const u32 c0 = threadIdx.x * per;
  u32 local = 0;
  for (u32 i = 0; i < per; ++i) {
    const u32 c = c0 + i;
    if (c < C) for (u32 s = 0; s < kSegs; ++s) local += part[u64(s) * C + c];
  }
  ws[threadIdx.x] = local;
  __syncthreads();
  for (u32 d = 1; d < 1024; d <<= 1) {
    const u32 v = threadIdx.x >= d ? ws[threadIdx.x - d] : 0;
    __syncthreads();
    ws[threadIdx.x] += v;
    __syncthreads();
  }
  u32 run = ws[threadIdx.x] - local;
  for (u32 i = 0; i < per; ++i) {
    const u32 c = c0 + i;
    if (c >= C) break;
    base[c] = run;
    for (u32 s = 0; s < kSegs; ++s) {
      const u32 p = part[u64(s) * C + c];
      part[u64(s) * C + c] = run;
      run += p;
    }
  }
  if (threadIdx.x == 1023) base[C] = run;
}

__global__ void k_scan_c(u32* __restrict__ H, u32 C, const u32* __restrict__ part) {
  const u32 c = blockIdx.x * blockDim.x + threadIdx.x;
  const u32 s = blockIdx.y;
  if (c >= C) return;
  const u32 per = kTiles / kSegs;
  u32 v[kTiles / kSegs];
#pragma unroll
  for (u32 i = 0; i < per; ++i) v[i] = H[u64(s * per + i) * C + c];
  u32 run = part[u64(s) * C + c];
#pragma unroll
  for (u32 i = 0; i < per; ++i) {
    H[u64(s * per + i) * C + c] = run;
    run += v[i];
  }
}

struct Rec { u64 a, b; };

template <bool AOS>
__global__ __launch_bounds__(kBlock) void k_scatter(const u32* __restrict__ grp, const uint8_t* __restrict__ flags,
                                                    const u64* __restrict__ idx, const u64* __restrict__ term,
                                                    u64 M, u32 C, u32 T, const u32* __restrict__ B,
                                                    u64* __restrict__ out_a, u64* __restrict__ out_b) {
  extern __shared__ u32 h[];
  const u32* row = B + u64(blockIdx.x) * C;
  for (u32 c = threadIdx.x; c < C; c += kBlock) h[c] = row[c];
  __syncthreads();
  const u64 t0 = u64(blockIdx.x) * T;
  const u64 t1 = t0 + T < M ? t0 + T : M;
  for (u64 j0 = t0 + threadIdx.x; j0 < t1; j0 += kBlock * 4) {
    u32 g[4];
    u64 ix[4], tm[4];
    uint8_t f[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const u64 j = j0 + u64(k) * kBlock;
      const bool live = j < t1;
      const u64 jj = live ? j : t0;
      g[k] = grp[jj];
      ix[k] = idx[jj];
      tm[k] = term[jj];
      f[k] = flags[jj];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const u64 j = j0 + u64(k) * kBlock;
      if (j >= t1) continue;
      const u32 pos = atomicAdd(&h[g[k] >> kChunkShift], 1u);
      const u64 mr = u64(g[k] & 511u) | (u64(f[k]) << 17) | (u64(u32(tm[k])) << 32);
      if (AOS) {
        Rec* o = reinterpret_cast<Rec*>(out_a);
        o[pos] = Rec{ix[k], mr};
      } else {
        out_a[pos] = ix[k];
        out_b[pos] = mr;
      }
    }
  }
}

int main() {
  const u64 M = 1ull << 24, G = 1ull << 24;
  const u32 C = u32(G >> kChunkShift);
  const u32 T = u32(M / kTiles);
  std::vector<u32> hg(M);
  for (u64 i = 0; i < M; ++i) hg[i] = u32(i);
  std::mt19937_64 rng(7);
  std::shuffle(hg.begin(), hg.end(), rng);
  u32 *grp, *H, *part, *base;
  uint8_t* flags;
  u64 *idx, *term, *oa, *ob;
  CK(hipMalloc(&grp, M * 4));
  CK(hipMalloc(&flags, M));
  CK(hipMalloc(&idx, M * 8));
  CK(hipMalloc(&term, M * 8));
  CK(hipMalloc(&oa, M * 16));
  CK(hipMalloc(&ob, M * 8));
  CK(hipMalloc(&H, u64(kTiles) * C * 4));
  CK(hipMalloc(&part, u64(kSegs) * C * 4));
  CK(hipMalloc(&base, (C + 1) * 4));
  CK(hipMemcpy(grp, hg.data(), M * 4, hipMemcpyHostToDevice));
  CK(hipMemset(flags, 1, M));
  CK(hipMemset(idx, 3, M * 8));
  CK(hipMemset(term, 0, M * 8));
  CK(hipFuncSetAttribute((const void*)k_hist, hipFuncAttributeMaxDynamicSharedMemorySize, C * 4));
  CK(hipFuncSetAttribute((const void*)k_scatter<true>, hipFuncAttributeMaxDynamicSharedMemorySize, C * 4));
  CK(hipFuncSetAttribute((const void*)k_scatter<false>, hipFuncAttributeMaxDynamicSharedMemorySize, C * 4));
  hipEvent_t e[6];
  for (auto& x : e) CK(hipEventCreate(&x));
  const int reps = 30;
  float th = 0, ts = 0, tA = 0, tS = 0;
  for (int r = 0; r < reps + 3; ++r) {
    CK(hipEventRecord(e[0]));
    hipLaunchKernelGGL(k_hist, dim3(kTiles), dim3(kBlock), C * 4, 0, grp, M, C, T, H);
    CK(hipEventRecord(e[1]));
    hipLaunchKernelGGL(k_scan_a, dim3(C / 256, kSegs), dim3(256), 0, 0, H, C, part);
    hipLaunchKernelGGL(k_scan_b, dim3(1), dim3(1024), 0, 0, part, C, base);
    hipLaunchKernelGGL(k_scan_c, dim3(C / 256, kSegs), dim3(256), 0, 0, H, C, part);
    CK(hipEventRecord(e[2]));
    hipLaunchKernelGGL(k_scatter<true>, dim3(kTiles), dim3(kBlock), C * 4, 0, grp, flags, idx, term, M, C, T,
                       H, oa, ob);
    CK(hipEventRecord(e[3]));
    hipLaunchKernelGGL(k_scatter<false>, dim3(kTiles), dim3(kBlock), C * 4, 0, grp, flags, idx, term, M, C, T,
                       H, oa, ob);
    CK(hipEventRecord(e[4]));
    CK(hipEventSynchronize(e[4]));
    float a, b, c, d;
    CK(hipEventElapsedTime(&a, e[0], e[1]));
    CK(hipEventElapsedTime(&b, e[1], e[2]));
    CK(hipEventElapsedTime(&c, e[2], e[3]));
    CK(hipEventElapsedTime(&d, e[3], e[4]));
    if (r >= 3) { th += a; ts += b; tA += c; tS += d; }
  }
  CK(hipGetLastError());
  // check: base is the chunk-count exclusive scan (every chunk holds 512 records)
  std::vector<u32> hb(C + 1);
  CK(hipMemcpy(hb.data(), base, (C + 1) * 4, hipMemcpyDeviceToHost));
  bool ok = hb[C] == M;
  for (u32 c = 0; c < C && ok; ++c) ok = hb[c] == c * 512u;
  // check: the SoA output's mr low bits are groups of their chunk
  std::vector<u64> hm(M);
  CK(hipMemcpy(hm.data(), ob, M * 8, hipMemcpyDeviceToHost));
  std::vector<u32> seen(C * 512, 0);
  for (u32 c = 0; c < C && ok; ++c)
    for (u32 i = hb[c]; i < hb[c + 1]; ++i) seen[c * 512 + (hm[i] & 511)]++;
  for (u64 g = 0; g < G && ok; ++g) ok = seen[g] == 1;
  printf("{\"hist_us\": %.1f, \"scan_us\": %.1f, \"scatter_aos16_us\": %.1f, \"scatter_soa_us\": %.1f, \"ok\": %s}\n",
         th * 1e3 / reps, ts * 1e3 / reps, tA * 1e3 / reps, tS * 1e3 / reps, ok ? "true" : "false");
  return ok ? 0 : 2;
}
