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
extern "C" int fence_launch(int kind, int nblk, int* sink, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (kind == 0) hipLaunchKernelGGL(acq_kernel, dim3(nblk), dim3(64), 0, s, sink);
  else if (kind == 1) hipLaunchKernelGGL(rel_kernel, dim3(nblk), dim3(64), 0, s, sink);
  else hipLaunchKernelGGL(acqsys_kernel, dim3(nblk), dim3(64), 0, s, sink);
  return (int)hipGetLastError();
}
