// calib.hip -- the HBM ceiling the roofline fractions are also reported against (bench.py
// roofline.measured): a streaming copy (read + write, the shape of the NFA kernels' traffic) and a
// streaming read over buffers far larger than the 256 MB MALL, 16-B vector accesses, grid-stride over
// 8 or 32 workgroups of 256 per CU (or one element per thread), several launches timed with HIP
// events, the best kept.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

__global__ __launch_bounds__(256) void copy_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    const uint4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
    dst[i] = a;
    dst[i + stride] = b;
    dst[i + 2 * stride] = c;
    dst[i + 3 * stride] = d;
  }
  for (; i < n; i += stride) dst[i] = src[i];
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void copy1_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src) + i);
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(dst) + i);
  }
}

__global__ __launch_bounds__(256) void read_kernel(const uint4* __restrict__ src, int64_t n, uint32_t* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  for (; i + 3 * stride < n; i += 4 * stride) {
    const uint4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
    acc ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c.x ^ c.y ^ c.z ^ c.w ^ d.x ^ d.y ^ d.z ^ d.w;
  }
  for (; i < n; i += stride) acc ^= src[i].x ^ src[i].y ^ src[i].z ^ src[i].w;
  if (acc == 0x9E3779B9u) out[0] = acc;  // (keeps the loads; practically never stores)
}

}  // namespace

// Best-of-`iters` streaming copy and read bandwidth (GB/s of bytes moved: copy counts read + write)
// over `bytes`-sized buffers on `device`.
extern "C" int sdh_calibrate_hbm(int32_t device, int64_t bytes, int32_t iters, double* copy_gbps, double* read_gbps) {
  if (bytes < (1 << 20) || iters < 1 || !copy_gbps || !read_gbps) return -1;
  if (hipSetDevice(device) != hipSuccess) return -3;
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
  const int64_t n = bytes / 16;
  uint4 *a = nullptr, *b = nullptr;
  uint32_t* o = nullptr;
  int rc = 0;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  hipStream_t s = nullptr;
  if (hipMalloc(&a, n * 16) != hipSuccess || hipMalloc(&b, n * 16) != hipSuccess || hipMalloc(&o, 4) != hipSuccess ||
      hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess ||
      hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
    rc = -3;
  } else {
    (void)hipMemsetAsync(a, 1, n * 16, s);
    (void)hipMemsetAsync(b, 0, n * 16, s);
    const dim3 block(256);
    float best_c = 1e30f, best_r = 1e30f;
    auto timed = [&](auto launch) {
      float ms = 0;
      (void)hipEventRecord(e0, s);
      launch();
      (void)hipEventRecord(e1, s);
      (void)hipEventSynchronize(e1);
      (void)hipEventElapsedTime(&ms, e0, e1);
      return ms;
    };
    // grid-stride at 8 / 32 workgroups per CU, and one element per thread with nontemporal stores:
    // the best of them is the ceiling
    for (int it = 0; it < iters + 1; ++it) {  // (the first round warms up)
      for (int per_cu : {8, 32}) {
        const dim3 grid(cus * per_cu);
        const float c = timed([&] { hipLaunchKernelGGL(copy_kernel, grid, block, 0, s, a, b, n); });
        const float r = timed([&] { hipLaunchKernelGGL(read_kernel, grid, block, 0, s, a, n, o); });
        if (it) {
          best_c = c < best_c ? c : best_c;
          best_r = r < best_r ? r : best_r;
        }
      }
      const dim3 g1((unsigned)((n + 255) / 256));
      const float c1 = timed([&] { hipLaunchKernelGGL(copy1_kernel, g1, block, 0, s, a, b, n); });
      if (it) best_c = c1 < best_c ? c1 : best_c;
    }
    if (hipGetLastError() != hipSuccess) rc = -3;
    *copy_gbps = 2.0 * (double)n * 16 / (best_c * 1e-3) / 1e9;
    *read_gbps = (double)n * 16 / (best_r * 1e-3) / 1e9;
  }
  if (s) (void)hipStreamSynchronize(s);
  if (a) (void)hipFree(a);
  if (b) (void)hipFree(b);
  if (o) (void)hipFree(o);
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  if (s) (void)hipStreamDestroy(s);
  return rc;
}
