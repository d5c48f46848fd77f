// valu_bench.hip -- issue cost of the forward epilogue's vector instructions on one MI355X:
// 1024 blocks x 256 threads (4 waves per SIMD on 256 CUs), each wave running ITER rounds of 16
// independent copies of one instruction form; prints cycles per wave-instruction per SIMD.
//   hipcc --offload-arch=gfx950 -O3 -o valu_bench tools/valu_bench.hip && ./valu_bench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

constexpr int ITER = 2048;

#define REP16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

template <int MODE>
__global__ __launch_bounds__(256) void bench(int* out, int seed) {
  int v[16];
  float f[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    v[q] = (int)threadIdx.x * 7 + q + seed;
    f[q] = (float)v[q];
  }
  const int thr = seed + 100, tlo = seed - 100;
  for (int it = 0; it < ITER; ++it) {
    if (MODE == 0) {  // v_add_f32 (VOP2)
#define X(q) asm volatile("v_add_f32_e32 %0, %0, %1" : "+v"(f[q]) : "v"(f[(q + 1) & 15]));
      REP16(X)
#undef X
    } else if (MODE == 1) {  // v_cmp_ge_i32_e64 -> SGPR pair
#define X(q)                                                              \
  {                                                                       \
    uint64_t m;                                                           \
    asm volatile("v_cmp_ge_i32_e64 %0, %1, %2" : "=s"(m) : "v"(v[q]), "v"(thr)); \
  }
      REP16(X)
#undef X
    } else if (MODE == 2) {  // v_cndmask_b32_e64 with an SGPR mask
      uint64_t m = 0x5555555555555555ull ^ (uint64_t)it;
#define X(q) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(f[q]) : "v"(f[(q + 3) & 15]), "s"(m));
      REP16(X)
#undef X
    } else if (MODE == 3) {  // v_addc_co_u32_e64 (shift-in of a mask bit)
      uint64_t m = 0x5555555555555555ull ^ (uint64_t)it;
#define X(q)                                                                         \
  {                                                                                  \
    uint64_t co;                                                                     \
    asm volatile("v_addc_co_u32_e64 %0, %1, %0, %0, %2" : "+v"(v[q]), "=s"(co) : "s"(m)); \
  }
      REP16(X)
#undef X
    } else if (MODE == 4) {  // v_cmp_e64 then v_cndmask on its mask (dependent pair)
#define X(q)                                                                                              \
  {                                                                                                       \
    uint64_t m;                                                                                           \
    asm volatile("v_cmp_ge_i32_e64 %1, %2, %3\n\tv_cndmask_b32_e64 %0, %0, %4, %1"                       \
                 : "+v"(f[q]), "=&s"(m) : "v"(v[q]), "v"(thr), "v"(f[(q + 5) & 15]));                     \
  }
      REP16(X)
#undef X
    } else if (MODE == 5) {  // v_sub_u32 (VOP2 int)
#define X(q) asm volatile("v_sub_u32_e32 %0, %0, %1" : "+v"(v[q]) : "v"(v[(q + 1) & 15]));
      REP16(X)
#undef X
    } else if (MODE == 6) {  // v_med3_i32 (VOP3)
#define X(q) asm volatile("v_med3_i32 %0, %0, %1, %2" : "+v"(v[q]) : "v"(tlo), "v"(thr));
      REP16(X)
#undef X
    } else if (MODE == 7) {  // v_cmp_ge_i32_e32 -> VCC then v_cndmask_b32_e32 (VCC)
#define X(q)                                                                                  \
  asm volatile("v_cmp_ge_i32_e32 vcc, %1, %2\n\tv_cndmask_b32_e32 %0, %0, %3, vcc"            \
               : "+v"(f[q]) : "v"(v[q]), "v"(thr), "v"(f[(q + 5) & 15]) : "vcc");
      REP16(X)
#undef X
    } else if (MODE == 8) {  // v_pk_add_f32 (2 fp32 per lane)
#define X(q)                                                                                        \
  {                                                                                                 \
    typedef float f2 __attribute__((ext_vector_type(2)));                                           \
    f2 a = {f[q], f[(q + 1) & 15]}, b = {f[(q + 2) & 15], f[(q + 3) & 15]};                          \
    asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a) : "v"(b));                                     \
    f[q] = a.x;                                                                                     \
  }
      REP16(X)
#undef X
    } else if (MODE == 10 || MODE == 11) {  // one ps of the forward's ternary ADC: 10 instructions
      // 10: SGPR masks, VOP3 forms (cimq_part_dense.hip adc_ps); 11: VCC, VOP2 / VOPC forms
#pragma unroll
      for (int q = 0; q < 16; q += 4) {
        const int ps = v[q], pz = v[q + 1], span = v[q + 2], cf = __float_as_int(f[q + 3]);
        float& acc = f[q];
        uint32_t& sp = reinterpret_cast<uint32_t&>(v[q + 1]);
        uint32_t& shi = reinterpret_cast<uint32_t&>(v[q + 2]);
        uint32_t& slo = reinterpret_cast<uint32_t&>(v[q + 3]);
        float a;
        int t;
        if (MODE == 10) {
          uint64_t mh, ml, mp, co;
          asm volatile(
              "v_sub_u32_e32 %[t], %[ps], %[pz]\n\t"
              "v_cmp_ge_i32_e64 %[mh], %[ps], %[thi]\n\t"
              "v_cmp_le_i32_e64 %[ml], %[ps], %[tlo]\n\t"
              "v_cmp_le_u32_e64 %[mp], %[t], %[span]\n\t"
              "v_cndmask_b32_e64 %[a], 0, %[cf], %[mh]\n\t"
              "v_cndmask_b32_e64 %[a], %[a], -%[cf], %[ml]\n\t"
              "v_add_f32_e32 %[acc], %[acc], %[a]\n\t"
              "v_addc_co_u32_e64 %[sp], %[co], %[sp], %[sp], %[mp]\n\t"
              "v_addc_co_u32_e64 %[shi], %[co], %[shi], %[shi], %[mh]\n\t"
              "v_addc_co_u32_e64 %[slo], %[co], %[slo], %[slo], %[ml]"
              : [mh] "=&s"(mh), [ml] "=&s"(ml), [mp] "=&s"(mp), [co] "=&s"(co), [a] "=&v"(a), [t] "=&v"(t),
                [acc] "+v"(acc), [sp] "+v"(sp), [shi] "+v"(shi), [slo] "+v"(slo)
              : [ps] "v"(ps), [pz] "v"(pz), [thi] "v"(thr), [tlo] "v"(tlo), [span] "v"(span), [cf] "v"(cf));
        } else {
          const int ncf = cf ^ (int)0x80000000;
          asm volatile(
              "v_sub_u32_e32 %[t], %[ps], %[pz]\n\t"
              "v_cmp_ge_i32_e32 vcc, %[ps], %[thi]\n\t"
              "v_cndmask_b32_e32 %[a], 0, %[cf], vcc\n\t"
              "v_addc_co_u32_e32 %[shi], vcc, %[shi], %[shi], vcc\n\t"
              "v_cmp_le_i32_e32 vcc, %[ps], %[tlo]\n\t"
              "v_cndmask_b32_e32 %[a], %[a], %[ncf], vcc\n\t"
              "v_addc_co_u32_e32 %[slo], vcc, %[slo], %[slo], vcc\n\t"
              "v_add_f32_e32 %[acc], %[acc], %[a]\n\t"
              "v_cmp_le_u32_e32 vcc, %[t], %[span]\n\t"
              "v_addc_co_u32_e32 %[sp], vcc, %[sp], %[sp], vcc"
              : [a] "=&v"(a), [t] "=&v"(t), [acc] "+v"(acc), [sp] "+v"(sp), [shi] "+v"(shi), [slo] "+v"(slo)
              : [ps] "v"(ps), [pz] "v"(pz), [thi] "v"(thr), [tlo] "v"(tlo), [span] "v"(span), [cf] "v"(cf),
                [ncf] "v"(ncf)
              : "vcc");
        }
      }
    } else if (MODE == 9) {  // v_lshl_or_b32 (VOP3 int, the shift-in without masks)
#define X(q) asm volatile("v_lshl_or_b32 %0, %0, 1, %1" : "+v"(v[q]) : "v"(v[(q + 2) & 15]));
      REP16(X)
#undef X
    }
  }
  int acc = 0;
#pragma unroll
  for (int q = 0; q < 16; ++q) acc += v[q] + (int)f[q];
  if (acc == 0x7fffffff) out[threadIdx.x] = acc;
}

static int g_blocks = 1024;

template <int MODE>
float run(int* d, int per_iter, const char* name) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(bench<MODE>, dim3(g_blocks), dim3(256), 0, 0, d, 1);
  hipEventRecord(a);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(bench<MODE>, dim3(g_blocks), dim3(256), 0, 0, d, r);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  ms /= 5;
  // per SIMD: 4 waves x ITER x per_iter instructions; 2.4 GHz
  const double instr = (g_blocks / 256.0) * ITER * per_iter;
  const double cyc = ms * 1e-3 * 2.4e9;
  printf("%-34s %8.3f ms  %6.2f cycles / wave-instruction / SIMD\n", name, ms, cyc / instr);
  return ms;
}

int main(int argc, char** argv) {
  int* d;
  hipMalloc(&d, 4096);
  if (argc > 1) g_blocks = atoi(argv[1]);
  printf("%d blocks of 4 waves: %.1f waves per SIMD\n", g_blocks, g_blocks / 256.0);
  run<0>(d, 16, "v_add_f32_e32");
  run<5>(d, 16, "v_sub_u32_e32");
  run<1>(d, 16, "v_cmp_ge_i32_e64 (sgpr)");
  run<2>(d, 16, "v_cndmask_b32_e64 (sgpr mask)");
  run<3>(d, 16, "v_addc_co_u32_e64 (sgpr carry)");
  run<4>(d, 32, "v_cmp_e64 + v_cndmask_e64 pair");
  run<7>(d, 32, "v_cmp_e32 + v_cndmask_e32 (vcc)");
  run<6>(d, 16, "v_med3_i32");
  run<8>(d, 16, "v_pk_add_f32");
  run<9>(d, 16, "v_lshl_or_b32");
  run<10>(d, 40, "ADC ps: SGPR masks, VOP3 (x10 instr)");
  run<11>(d, 40, "ADC ps: VCC, VOP2/VOPC (x10 instr)");
  hipFree(d);
  return 0;
}
