// VALU issue-rate probe for gfx950 (tool only): wave64 cycles per instruction
// for the instruction kinds the median kernels are made of, by waves per SIMD.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/_build/valu_rate_probe tools/valu_rate_probe.hip
//   tools/_build/valu_rate_probe
//
// Each wave runs ITER x 64 instructions of one kind over 16 independent
// registers (dependency distance 16, so latency never stalls the stream).
// Blocks of 256 lanes (one wave per SIMD); W blocks per CU give W waves per
// SIMD.  Cycles per instruction per SIMD = elapsed x clock x 1024 SIMDs /
// (waves x instructions): at one wave per SIMD it is the single-wave issue
// cost, at 2+ waves per SIMD the SIMD's own rate.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define R16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

constexpr int ITER = 2048;

template <int KIND>
__global__ __launch_bounds__(256) void probe(float* out, float seed) {
  float a[16];
  double a2[8];
  uint64_t cm[4] = {0, 0, 0, 0};
  const uint64_t msk = 0x5555aaaa3333ccccull ^ blockIdx.x;
  uint32_t b = threadIdx.x * 0x9e3779b9u;
#pragma unroll
  for (int i = 0; i < 16; ++i) a[i] = seed * (threadIdx.x + i);
#pragma unroll
  for (int i = 0; i < 8; ++i) a2[i] = seed * (threadIdx.x + i);
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int rep = 0; rep < 4; ++rep) {
#define OP(i)                                                                                                        \
  if constexpr (KIND == 0) asm volatile("v_max_f32 %0, %0, %1" : "+v"(a[i]) : "v"(a[(i + 1) & 15]));                 \
  if constexpr (KIND == 1) asm volatile("v_pk_max_i16 %0, %0, %1" : "+v"(a[i]) : "v"(a[(i + 1) & 15]));              \
  if constexpr (KIND == 2) asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(a[(i + 1) & 15]), "v"(a[(i + 2) & 15])); \
  if constexpr (KIND == 3) asm volatile("v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "=v"(a[i]) : "v"(a[(i + 8) & 15])); \
  if constexpr (KIND == 4) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(a[(i + 1) & 15]), "v"(a[(i + 2) & 15])); \
  if constexpr (KIND == 5) asm volatile("v_pk_max_f16 %0, %0, %1" : "+v"(a[i]) : "v"(a[(i + 1) & 15]));              \
  if constexpr (KIND == 6) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(a[(i + 1) & 15]) : "vcc"); \
  if constexpr (KIND == 7) asm volatile("v_pk_maximum3_f16 %0, %0, %1, %2" : "+v"(a[i]) : "v"(a[(i + 1) & 15]), "v"(a[(i + 2) & 15])); \
  if constexpr (KIND == 8) asm volatile("v_max_i16_sdwa %0, %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1" : "+v"(a[i]) : "v"(a[(i + 1) & 15])); \
  if constexpr (KIND == 9) asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(a[(i + 1) & 15]), "v"(a[(i + 2) & 15])); \
  if constexpr (KIND == 10) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[i]) : "v"(a[(i + 1) & 15]));                \
  if constexpr (KIND == 11) asm volatile("v_pk_min_i16 %0, %0, %1 op_sel:[0,1] op_sel_hi:[1,0]" : "+v"(a[i]) : "v"(a[(i + 1) & 15])); \
  if constexpr (KIND == 12) asm volatile("v_min_i32 %0, %0, %1" : "+v"(a[i]) : "v"(a[(i + 1) & 15])); \
  if constexpr (KIND == 13) asm volatile("v_min_u32 %0, %0, %1" : "+v"(a[i]) : "v"(a[(i + 1) & 15])); \
  if constexpr (KIND == 14) asm volatile("v_med3_i32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(a[(i + 1) & 15]), "v"(a[(i + 2) & 15])); \
  if constexpr (KIND == 15) asm volatile("v_min_i16 %0, %0, %1" : "+v"(a[i]) : "v"(a[(i + 1) & 15])); \
  if constexpr (KIND == 16) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(a[i]) : "v"(a[(i + 1) & 15])); \
  if constexpr (KIND == 17) asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(a[i])); \
  if constexpr (KIND == 18) asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(a[(i + 1) & 15]), "v"(a[(i + 2) & 15])); \
  if constexpr (KIND == 19) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xca" : "+v"(a[i]) : "v"(a[(i + 1) & 15]), "v"(a[(i + 2) & 15])); \
  if constexpr (KIND == 20) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a[i]) : "v"(a[(i + 1) & 15]), "s"(msk)); \
  if constexpr (KIND == 21) asm volatile("v_cmp_lt_u32_e64 %0, %1, %2" : "=s"(cm[i & 3]) : "v"(a[i]), "v"(a[(i + 1) & 15])); \
  if constexpr (KIND == 22) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(a[(i + 1) & 15]), "v"(a[(i + 2) & 15])); \
  if constexpr (KIND == 23) asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(a[i]), "+v"(a[(i + 8) & 15])); \
  if constexpr (KIND == 24) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(a[(i + 1) & 15])); \
  if constexpr (KIND == 25) asm volatile("v_pk_fma_f32 %0, %0, %1, %0" : "+v"(a2[i & 7]) : "v"(a2[(i + 1) & 7])); \
  if constexpr (KIND == 26) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[i]) : "v"(a[(i + 1) & 15])); \
  if constexpr (KIND == 27) asm volatile("v_max_u16 %0, %0, %1" : "+v"(a[i]) : "v"(a[(i + 1) & 15])); \
  if constexpr (KIND == 28) asm volatile("v_minimum3_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(a[(i + 1) & 15]), "v"(a[(i + 2) & 15])); \
  if constexpr (KIND == 29) asm volatile("v_min3_u32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(a[(i + 1) & 15]), "v"(a[(i + 2) & 15])); \
  if constexpr (KIND == 30) asm volatile("v_dot2_u32_u16 %0, %1, %2, %0" : "+v"(a[i]) : "v"(a[(i + 1) & 15]), "v"(a[(i + 2) & 15])); \
  if constexpr (KIND == 31) asm volatile("v_and_b32 %0, %0, %1" : "+v"(a[i]) : "v"(a[(i + 1) & 15])); \
  if constexpr (KIND == 32) asm volatile("v_sad_u8 %0, %1, %2, %0" : "+v"(a[i]) : "v"(a[(i + 1) & 15]), "v"(a[(i + 2) & 15])); \
  if constexpr (KIND == 33) asm volatile("v_sad_u16 %0, %1, %2, %0" : "+v"(a[i]) : "v"(a[(i + 1) & 15]), "v"(a[(i + 2) & 15])); \
  if constexpr (KIND == 34) asm volatile("v_sad_hi_u8 %0, %1, %2, %0" : "+v"(a[i]) : "v"(a[(i + 1) & 15]), "v"(a[(i + 2) & 15])); \
  if constexpr (KIND == 35) asm volatile("v_msad_u8 %0, %1, %2, %0" : "+v"(a[i]) : "v"(a[(i + 1) & 15]), "v"(a[(i + 2) & 15])); \
  if constexpr (KIND == 36) asm volatile("v_pk_ashrrev_i16 %0, 15, %0" : "+v"(a[i])); \
  if constexpr (KIND == 37) asm volatile("v_pk_max_u16 %0, %0, %1" : "+v"(a[i]) : "v"(a[(i + 1) & 15])); \
  if constexpr (KIND == 38) asm volatile("v_sad_u32 %0, %1, %2, %0" : "+v"(a[i]) : "v"(a[(i + 1) & 15]), "v"(a[(i + 2) & 15])); \
  if constexpr (KIND == 39) asm volatile("v_add_u32_dpp %0, %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(a[i]) : "v"(a[(i + 8) & 15])); \
  if constexpr (KIND == 40) asm volatile("v_lshl_or_b32 %0, %0, 8, %1" : "+v"(a[i]) : "v"(a[(i + 1) & 15])); \
  if constexpr (KIND == 41) asm volatile("v_bcnt_u32_b32 %0, %1, %0" : "+v"(a[i]) : "v"(a[(i + 1) & 15])); \
  if constexpr (KIND == 42) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(a[(i + 1) & 15]), "v"(a[(i + 2) & 15])); \
  if constexpr (KIND == 43) asm volatile("v_sub_u16 %0, %0, %1" : "+v"(a[i]) : "v"(a[(i + 1) & 15]));
      R16(OP)
#undef OP
    }
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += a[i];
  s += __uint_as_float(b);
#pragma unroll
  for (int i = 0; i < 8; ++i) s += float(a2[i]);
  s += float(cm[0] ^ cm[1] ^ cm[2] ^ cm[3]);
  if (s == 1.2345f) out[threadIdx.x] = s;  // keep the work
}

static const char* kNames[] = {"v_max_f32", "v_pk_max_i16", "v_med3_f32", "v_mov_b32_dpp", "v_fma_f32",
                               "v_pk_max_f16", "v_cndmask_b32", "v_pk_maximum3_f16", "v_max_i16_sdwa",
                               "v_max3_f32", "v_xor_b32", "v_pk_min_i16 op_sel", "v_min_i32", "v_min_u32", "v_med3_i32", "v_min_i16", "v_sub_u32", "v_lshrrev_b32", "v_bfi_b32", "v_bitop3_b32", "v_cndmask_b32 sgpr", "v_cmp_lt_u32", "v_perm_b32", "v_permlane32_swap", "v_add_f32", "v_pk_fma_f32", "v_pk_add_u16", "v_max_u16", "v_minimum3_f32", "v_min3_u32", "v_dot2_u32_u16", "v_and_b32", "v_sad_u8", "v_sad_u16", "v_sad_hi_u8", "v_msad_u8", "v_pk_ashrrev_i16", "v_pk_max_u16", "v_sad_u32", "v_add_u32_dpp", "v_lshl_or_b32", "v_bcnt_u32_b32", "v_add3_u32", "v_sub_u16"};

template <int KIND>
float run(int blocks, float* out) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(probe<KIND>, dim3(blocks), dim3(256), 0, 0, out, 1.0f);
  hipEventRecord(e0);
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(probe<KIND>, dim3(blocks), dim3(256), 0, 0, out, 1.0f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / 3;
}

template <int KIND>
void row(float* out, int cus, double ghz) {
  printf("%-22s", kNames[KIND]);
  for (int w : {1, 2, 3, 4, 8}) {
    const int blocks = cus * w;
    const float ms = run<KIND>(blocks, out);
    const double insts = double(blocks) * 4 * ITER * 64;  // wave-instructions
    const double cyc = ms * 1e-3 * ghz * 1e9 * cus * 4 / insts;
    printf("  W=%d %5.2f", w, cyc);
  }
  printf("   (cycles per wave64 instruction per SIMD)\n");
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  const double ghz = p.clockRate / 1e6;
  printf("%s: %d CUs, clock %.3f GHz (cycles below at this clock)\n", p.gcnArchName, cus, ghz);
  float* out;
  hipMalloc(&out, 4096);
  row<0>(out, cus, ghz);
  row<4>(out, cus, ghz);
  if (getenv("VALU_PROBE_SAD")) {  // round 4: the counting-selection candidates only
    for (int w = 0; w < 1; ++w) {
      row<10>(out, cus, ghz);
      row<22>(out, cus, ghz);
      row<32>(out, cus, ghz);
      row<33>(out, cus, ghz);
      row<34>(out, cus, ghz);
      row<35>(out, cus, ghz);
      row<36>(out, cus, ghz);
      row<37>(out, cus, ghz);
      row<38>(out, cus, ghz);
      row<39>(out, cus, ghz);
      row<40>(out, cus, ghz);
      row<41>(out, cus, ghz);
      row<42>(out, cus, ghz);
      row<43>(out, cus, ghz);
    }
    hipFree(out);
    return 0;
  }
  row<12>(out, cus, ghz);
  row<13>(out, cus, ghz);
  row<14>(out, cus, ghz);
  row<15>(out, cus, ghz);
  row<16>(out, cus, ghz);
  row<17>(out, cus, ghz);
  row<18>(out, cus, ghz);
  row<19>(out, cus, ghz);
  row<20>(out, cus, ghz);
  row<21>(out, cus, ghz);
  row<22>(out, cus, ghz);
  row<23>(out, cus, ghz);
  row<24>(out, cus, ghz);
  row<25>(out, cus, ghz);
  row<26>(out, cus, ghz);
  row<27>(out, cus, ghz);
  row<28>(out, cus, ghz);
  row<29>(out, cus, ghz);
  row<30>(out, cus, ghz);
  row<31>(out, cus, ghz);
  hipFree(out);
  return 0;
}
