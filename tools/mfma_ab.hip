#include <hip/hip_runtime.h>
#include <stdio.h>
typedef unsigned int v4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));
// MODE 0: A in VGPR; 1: A in AGPR; 2: A in AGPR + one ds_read_b128 per 2 MFMAs (B from LDS, used at once)
// 3: one read per 2 MFMAs, 8 MFMAs ahead; 4: one read per MFMA, 8 ahead
// 14-21: memory operations among the MFMAs at the fused layer1 block's
// density (one VMEM instruction per 48 MFMAs per wave): 24 units of (one
// ds_read 6 ahead + 2 MFMAs) per iteration, one memory operation at unit 5
// (and one more at unit 17 in mode 19), vmcnt(8) at the iteration's end.
// 14: LDS-DMA piece (buffer_load_dwordx4 ... lds, 1 KB) from HBM (a wave-private
//     256 KB window of a 256 MB buffer, into an LDS area nothing reads)
// 15: as 14, MFMA-only units (no ds_read)
// 16: buffer_store_dwordx2 (512 B, wave-private 128 KB window)
// 17: as 14, the source window 16 KB per wave (L2-resident)
// 18: buffer_load_dwordx4 to VGPRs from HBM (consumed only after the loop)
// 19: DMA piece at unit 5 + store at unit 17
// 20: ds_write_b64 (512 B) instead
// 21: as 14 with a readlane -> SALU -> M0 address chain (as the kernel's)
template <int MODE>
__global__ __launch_bounds__(256, 1) void k(float* out, int iters, const char* gsrc, char* gdst) {
  __shared__ __attribute__((aligned(16))) char sm[65536];
  const int lane = threadIdx.x & 63;
  v4 w[8];
  for (int i = 0; i < 8; ++i) w[i] = (v4){(unsigned)(lane + i) * 0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u};
  v4 b = (v4){0x3c003c00u, 0x3c003c00u, 0x3c003c00u, (unsigned)lane};
  f4 acc[8];
  typedef float f16v __attribute__((ext_vector_type(16)));
  f16v acc16[2] = {};
  for (int i = 0; i < 8; ++i) acc[i] = (f4){0, 0, 0, 0};
  for (int i = 0; i < 1024; ++i) ((float*)sm)[(threadIdx.x * 1024 + i) & 16383] = (float)i;
  __syncthreads();
  v4 bq[8], bq12[12];
  for (int i = 0; i < 12; ++i) bq12[i] = *(const v4*)(sm + ((lane * 16 + i * 2048) & 65535));
  for (int i = 0; i < 8; ++i) bq[i] = *(const v4*)(sm + ((lane * 16 + i * 1024) & 65535));
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)gsrc, (short)0, 0x7FFFFFF0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rdst = __builtin_amdgcn_make_buffer_rsrc((void*)gdst, (short)0, 0x7FFFFFF0, 0x00020000);
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)sm;
  const int wave = threadIdx.x >> 6;
  const unsigned wbase = __builtin_amdgcn_readfirstlane(lds0 + 32768 + wave * 8192);
  // 256 MB source / destination: workgroup-and-wave private 1 MB windows
  const int gbase = (blockIdx.x * 4 + wave) << 18;
  v4 ld3[3] = {};
  for (int it = 0; it < iters; ++it) {
    if (MODE >= 14 && MODE <= 21) {
      typedef unsigned v2 __attribute__((ext_vector_type(2)));
      const int win = MODE == 17 ? 15 : 255;
      const int go = gbase + ((it & win) << 10) + lane * 16;
#pragma unroll
      for (int u = 0; u < 24; ++u) {
        const bool rd = MODE != 15;
        const v4 bb = rd ? bq[u % 6] : b;
        int ad = (lane * 16 + u * 1024 + it * 64) & 32767;
        if (rd) bq[u % 6] = *(const v4*)(sm + ad);
        if (u == 5 || (MODE == 19 && u == 17)) {
          if (MODE == 14 || MODE == 15 || MODE == 17 || (MODE == 19 && u == 5)) {
            asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %2, 0 offen lds"
                         :
                         : "v"(go), "s"(wbase + (it & 7) * 1024), "s"(rsrc)
                         : "memory", "m0");
          } else if (MODE == 21) {
            int sv = __builtin_amdgcn_readlane(ad, 15);
            asm volatile("s_add_i32 %0, %0, 0" : "+s"(sv));
            asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %2, 0 offen lds"
                         :
                         : "v"(go), "s"(wbase + ((sv >> 20) & 7) * 1024 + (it & 7) * 1024), "s"(rsrc)
                         : "memory", "m0");
          } else if (MODE == 16 || MODE == 19) {
            __builtin_amdgcn_raw_buffer_store_b64((v2){(unsigned)ad, (unsigned)u}, rdst, (go - lane * 16) / 2 + lane * 8, 0, 0);
          } else if (MODE == 18) {
            asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(ld3[it & 1]) : "v"(go), "s"(rsrc) : "memory");
          } else if (MODE == 20) {
            *(v2*)(sm + 32768 + ((lane * 8 + wave * 4096 + (it & 7) * 512) & 16383)) = (v2){(unsigned)ad, (unsigned)it};
          }
        }
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc[(2 * u) & 7]) : "a"(w[u & 7]), "v"(bb));
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc[(2 * u + 1) & 7]) : "a"(w[(u + 1) & 7]), "v"(bb));
      }
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      continue;
    }
    if (MODE == 11) {  // as 7 but reads 12 ahead
#pragma unroll
      for (int u = 0; u < 24; ++u) {
        const v4 bb = bq12[u % 12];
        const int ad = (lane * 16 + u * 1024 + it * 64) & 65535;
        bq12[u % 12] = *(const v4*)(sm + ad);
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc[(2 * u) & 7]) : "a"(w[u & 7]), "v"(bb));
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc[(2 * u + 1) & 7]) : "a"(w[(u + 1) & 7]), "v"(bb));
      }
      continue;
    }
    if (MODE == 12) {  // reads issued but never waited for (results unused): pure issue cost
#pragma unroll
      for (int u = 0; u < 12; ++u) {
        const int ad = (lane * 16 + u * 1024 + it * 64) & 65535;
        v4 junk;
        asm volatile("ds_read_b128 %0, %1" : "=v"(junk) : "v"(ad));
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc[(2 * u) & 7]) : "a"(w[u & 7]), "v"(b));
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc[(2 * u + 1) & 7]) : "a"(w[(u + 1) & 7]), "v"(b));
      }
      asm volatile("s_waitcnt lgkmcnt(0)");
      continue;
    }
    if (MODE == 13) {  // 2 independent VALU per 2 MFMAs, no reads
#pragma unroll
      for (int u = 0; u < 12; ++u) {
        int ad = lane + u;
        asm volatile("v_xor_b32 %0, 0x40, %0\n\tv_add_u32 %0, 1, %0" : "+v"(ad));
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc[(2 * u) & 7]) : "a"(w[u & 7]), "v"(b));
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc[(2 * u + 1) & 7]) : "a"(w[(u + 1) & 7]), "v"(b));
        if (ad == 12345678) out[0] = 1.f;
      }
      continue;
    }
    if (MODE == 9 || MODE == 10) {  // 32x32x16: 12 units of one read (6 ahead) + ONE MFMA; 10: + 2 VALU
#pragma unroll
      for (int u = 0; u < 12; ++u) {
        const v4 bb = bq[u % 6];
        int ad = (lane * 16 + u * 1024 + it * 64) & 65535;
        if (MODE == 10) asm volatile("v_xor_b32 %0, 0x40, %0\n\tv_add_u32 %0, 0, %0" : "+v"(ad));
        bq[u % 6] = *(const v4*)(sm + ad);
        asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc16[u & 1]) : "a"(w[u & 7]), "v"(bb));
      }
      continue;
    }
    if (MODE == 7 || MODE == 8) {  // 12 units: one read (6 ahead) + 2 MFMAs; 8: + 2 address VALU per read
#pragma unroll
      for (int u = 0; u < 12; ++u) {
        const v4 bb = bq[u % 6];
        int ad = (lane * 16 + u * 1024 + it * 64) & 65535;
        if (MODE == 8) asm volatile("v_xor_b32 %0, 0x40, %0\n\tv_add_u32 %0, 0, %0" : "+v"(ad));
        bq[u % 6] = *(const v4*)(sm + ad);
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc[(2 * u) & 7]) : "a"(w[u & 7]), "v"(bb));
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc[(2 * u + 1) & 7]) : "a"(w[(u + 1) & 7]), "v"(bb));
      }
      continue;
    }
    if (MODE == 5 || MODE == 6) {  // 5: 2 accumulators alternating, 6: 1 accumulator
#pragma unroll
      for (int i = 0; i < 8; ++i)
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc[MODE == 5 ? (i & 1) : 0]) : "a"(w[i]), "v"(b));
      continue;
    }
    if (MODE >= 3) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const v4 bb = bq[i];
        if ((i & 1) == 0 || MODE == 4) bq[i] = *(const v4*)(sm + ((lane * 16 + i * 1024 + it * 64) & 65535));
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc[i]) : "a"(w[i]), "v"(bb));
      }
      continue;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (MODE == 2 && (i & 1) == 0) {
        b = *(const v4*)(sm + ((lane * 16 + i * 1024 + it * 64) & 65535));
      }
      if (MODE == 0)
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc[i]) : "v"(w[i]), "v"(b));
      else
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc[i]) : "a"(w[i]), "v"(b));
    }
  }
  asm volatile("s_nop 15");
  float s = 0;
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  s += acc16[0][3] + acc16[1][5];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  s += (float)(ld3[0][0] + ld3[1][1] + ld3[2][2]);
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
int main() {
  float* out;
  hipMalloc(&out, 256 * 256 * 4);
  char *gsrc, *gdst;
  hipMalloc(&gsrc, 256u << 20);
  hipMalloc(&gdst, 256u << 20);
  hipMemset(gsrc, 0, 256u << 20);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 20000;
  for (int rep = 0; rep < 2; ++rep) {
    if (rep) printf("-- second round\n");
    for (int m = 0; m < 22; ++m) {
      hipEventRecord(e0);
      if (m == 0) hipLaunchKernelGGL(k<0>, dim3(256), dim3(256), 0, 0, out, iters, gsrc, gdst);
      if (m == 1) hipLaunchKernelGGL(k<1>, dim3(256), dim3(256), 0, 0, out, iters, gsrc, gdst);
      if (m == 2) hipLaunchKernelGGL(k<2>, dim3(256), dim3(256), 0, 0, out, iters, gsrc, gdst);
      if (m == 3) hipLaunchKernelGGL(k<3>, dim3(256), dim3(256), 0, 0, out, iters, gsrc, gdst);
      if (m == 4) hipLaunchKernelGGL(k<4>, dim3(256), dim3(256), 0, 0, out, iters, gsrc, gdst);
      if (m == 5) hipLaunchKernelGGL(k<5>, dim3(256), dim3(256), 0, 0, out, iters, gsrc, gdst);
      if (m == 6) hipLaunchKernelGGL(k<6>, dim3(256), dim3(256), 0, 0, out, iters, gsrc, gdst);
      if (m == 7) hipLaunchKernelGGL(k<7>, dim3(256), dim3(256), 0, 0, out, iters / 3, gsrc, gdst);
      if (m == 8) hipLaunchKernelGGL(k<8>, dim3(256), dim3(256), 0, 0, out, iters / 3, gsrc, gdst);
      if (m == 9) hipLaunchKernelGGL(k<9>, dim3(256), dim3(256), 0, 0, out, iters / 3, gsrc, gdst);
      if (m == 10) hipLaunchKernelGGL(k<10>, dim3(256), dim3(256), 0, 0, out, iters / 3, gsrc, gdst);
      if (m == 11) hipLaunchKernelGGL(k<11>, dim3(256), dim3(256), 0, 0, out, iters / 6, gsrc, gdst);
      if (m == 12) hipLaunchKernelGGL(k<12>, dim3(256), dim3(256), 0, 0, out, iters / 3, gsrc, gdst);
      if (m == 13) hipLaunchKernelGGL(k<13>, dim3(256), dim3(256), 0, 0, out, iters / 3, gsrc, gdst);
      if (m == 14) hipLaunchKernelGGL(k<14>, dim3(256), dim3(256), 0, 0, out, iters / 6, gsrc, gdst);
      if (m == 15) hipLaunchKernelGGL(k<15>, dim3(256), dim3(256), 0, 0, out, iters / 6, gsrc, gdst);
      if (m == 16) hipLaunchKernelGGL(k<16>, dim3(256), dim3(256), 0, 0, out, iters / 6, gsrc, gdst);
      if (m == 17) hipLaunchKernelGGL(k<17>, dim3(256), dim3(256), 0, 0, out, iters / 6, gsrc, gdst);
      if (m == 18) hipLaunchKernelGGL(k<18>, dim3(256), dim3(256), 0, 0, out, iters / 6, gsrc, gdst);
      if (m == 19) hipLaunchKernelGGL(k<19>, dim3(256), dim3(256), 0, 0, out, iters / 6, gsrc, gdst);
      if (m == 20) hipLaunchKernelGGL(k<20>, dim3(256), dim3(256), 0, 0, out, iters / 6, gsrc, gdst);
      if (m == 21) hipLaunchKernelGGL(k<21>, dim3(256), dim3(256), 0, 0, out, iters / 6, gsrc, gdst);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      // MFMAs per wave in 16x16x32 units (a 32x32x16 counts as 2)
      const double per = (m == 11 || m >= 14) ? (iters / 6) * 48.0 : m >= 7 ? (iters / 3) * 24.0 : iters * 8.0;
      printf("mode %d: %.3f ms, %.1f ns per MFMA per SIMD, %.0f TFLOP/s\n", m, ms, ms * 1e6 / per,
             256.0 * 4 * per * 16384 / ms / 1e9);
      if (hipGetLastError() != hipSuccess) return 1;
    }
  }
  return 0;
}
