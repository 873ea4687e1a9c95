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
