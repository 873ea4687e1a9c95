#include <hip/hip_runtime.h>
__global__ void acq_kernel(int* sink) {
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  if (sink && threadIdx.x == 0 && blockIdx.x == 0) sink[0] = 1;
}
__global__ void rel_kernel(int* sink) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  if (sink && threadIdx.x == 0 && blockIdx.x == 0) sink[0] = 1;
}
__global__ void acqsys_kernel(int* sink) {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "");
  if (sink && threadIdx.x == 0 && blockIdx.x == 0) sink[0] = 1;
}
// no fence: the same grid as a pure delay (separates timing from cache state)
__global__ void nop_kernel(int* sink) {
  if (sink && threadIdx.x == 0 && blockIdx.x == 0) sink[0] = 1;
}
// no fence, ~110 us of s_sleep per wave: a long pure delay
__global__ void spin_kernel(int* sink) {
  for (int i = 0; i < 32; ++i) __builtin_amdgcn_s_sleep(127);
  if (sink && threadIdx.x == 0 && blockIdx.x == 0) sink[0] = 1;
}
extern "C" int fence_launch(int kind, int nblk, int* sink, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (kind == 0) hipLaunchKernelGGL(acq_kernel, dim3(nblk), dim3(64), 0, s, sink);
  else if (kind == 1) hipLaunchKernelGGL(rel_kernel, dim3(nblk), dim3(64), 0, s, sink);
  else if (kind == 3) hipLaunchKernelGGL(nop_kernel, dim3(nblk), dim3(64), 0, s, sink);
  else if (kind == 4) hipLaunchKernelGGL(spin_kernel, dim3(nblk), dim3(64), 0, s, sink);
  else hipLaunchKernelGGL(acqsys_kernel, dim3(nblk), dim3(64), 0, s, sink);
  return (int)hipGetLastError();
}
// LDS traffic only, within the workgroup's own allocation: every thread
// rewrites and re-reads its dwords of `bytes` of dynamic LDS `iters` times (a
// co-residency probe with the stem's footprint, 81,696 B)
__global__ void lds_kernel(int* sink, int iters, int words) {
  extern __shared__ float sm[];
  float acc = 0.f;
  for (int it = 0; it < iters; ++it) {
    for (int i = threadIdx.x; i < words; i += blockDim.x) sm[i] = acc + (float)(i + it);
    __syncthreads();
    for (int i = threadIdx.x; i < words; i += blockDim.x) acc += sm[words - 1 - i];
    __syncthreads();
  }
  if (sink && acc == -1.f) sink[0] = 1;
}
extern "C" int lds_launch(int nblk, int bytes, int iters, void* stream) {
  (void)hipFuncSetAttribute((const void*)lds_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  hipLaunchKernelGGL(lds_kernel, dim3(nblk), dim3(256), bytes, (hipStream_t)stream, nullptr, iters, bytes / 4);
  return (int)hipGetLastError();
}

// Co-residency probes with the stem's LDS footprint (81,696 B dynamic): each
// exercises ONE feature of stem_bf16_kernel while touching only its own LDS.
// kind 0: ds_bpermute_b32 (the stem's wave-rotation exchange)
// kind 1: v_mfma_f32_16x16x32_bf16 chains on registers
// kind 2: DPP row shifts + v_pk_max_i16 (the stem's pooling)
// kind 3: all three interleaved
typedef float probe_f4 __attribute__((ext_vector_type(4)));
typedef __bf16 probe_b8 __attribute__((ext_vector_type(8)));
__global__ __launch_bounds__(256) void probe_kernel(int* sink, int kind, int iters) {
  extern __shared__ float sm[];
  const int lane = threadIdx.x & 63;
  float v = (float)threadIdx.x;
  probe_f4 acc = {0.f, 0.f, 0.f, 0.f};
  probe_b8 a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = (__bf16)(0.001f * (lane + i));
    b[i] = (__bf16)(0.002f * (lane - i));
  }
  sm[threadIdx.x] = v;
  __syncthreads();
  for (int it = 0; it < iters; ++it) {
    if (kind == 0 || kind == 3)
      v += __int_as_float(__builtin_amdgcn_ds_bpermute(((lane + 48) & 63) << 2, __float_as_int(v))) * 1e-3f;
    if (kind == 1 || kind == 3)
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
    if (kind == 2 || kind == 3) {
      int x = __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x101, 0xF, 0xF, true);
      uint32_t r;
      asm volatile("v_pk_max_i16 %0, %1, 0" : "=v"(r) : "v"(x));
      v += (float)(r & 7) * 1e-3f;
    }
  }
  sm[threadIdx.x] += v + acc[0] + acc[1] + acc[2] + acc[3];
  __syncthreads();
  if (sink && sm[threadIdx.x ^ 1] == -1.f) sink[0] = 1;
}
extern "C" int probe_launch(int nblk, int bytes, int kind, int iters, void* stream) {
  (void)hipFuncSetAttribute((const void*)probe_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  hipLaunchKernelGGL(probe_kernel, dim3(nblk), dim3(256), bytes, (hipStream_t)stream, nullptr, kind, iters);
  return (int)hipGetLastError();
}
