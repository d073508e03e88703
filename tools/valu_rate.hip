// Micro-benchmark: SIMD cost of the instruction forms the LC kernel is built from, on gfx950, as a
// function of waves per SIMD (round-4 design input).
//
// Each wave runs ITERS iterations of one asm block of 16 instructions over 8 registers, visited
// round-robin (a register is rewritten every 8 instructions, so a chain's dependency distance is 8
// instructions: issue cost, not latency, unless the row says "chain").  s_memtime / s_memrealtime
// around the loop give the wave's shader cycles and the clock.  A 100 ms spin kernel runs first so
// the clock has left its idle state.
//   SIMD cycles per instruction = wave cycles / (waves per SIMD x instructions per wave)
//   hipcc --offload-arch=gfx950 -O3 -o .tmp/valu_rate tools/valu_rate.hip && .tmp/valu_rate
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f2 __attribute__((ext_vector_type(2)));

#define R8 "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7])
#define P8 "+v"(p[0]), "+v"(p[1]), "+v"(p[2]), "+v"(p[3]), "+v"(p[4]), "+v"(p[5]), "+v"(p[6]), "+v"(p[7])
// 16 instructions: register k = i mod 8 (operand %k), second operand the register 4 earlier
#define BODY16(I) I(0, 4) I(1, 5) I(2, 6) I(3, 7) I(4, 0) I(5, 1) I(6, 2) I(7, 3) I(0, 4) I(1, 5) I(2, 6) I(3, 7) I(4, 0) I(5, 1) I(6, 2) I(7, 3)
#define S(x) #x
#define XS(x) S(x)

__global__ void spin_kernel(float* out, int n)
{
    float x = threadIdx.x;
    for (int i = 0; i < n; i++) x = x * 0.999f + 1.0f;
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

template <int K>
__global__ __launch_bounds__(256) void rate_kernel(float* out, unsigned long long* cyc, int iters)
{
    const int t = threadIdx.x;
    float a[8];
    f2 p[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        a[i] = 1.0f + 1e-7f * (t + i);
        p[i] = f2{a[i], a[i] + 0.5f};
    }
    const unsigned long long smask = 0x5555555555555555ull;
    const unsigned vmask = (t & 1) ? 0xffffffffu : 0u;
    if constexpr (K == 22) asm volatile("s_mov_b32 vcc_lo, 0x55555555\n\ts_mov_b32 vcc_hi, 0x55555555" ::: "vcc");
    __shared__ float lds[4096];
    lds[t] = a[0];
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; it++) {
        if constexpr (K == 0) {
#define I(k, j) "v_mul_f32 %" #k ", %" #k ", %" #j "\n\t"
            asm volatile(BODY16(I) : R8);
#undef I
        } else if constexpr (K == 1) {
#define I(k, j) "v_pk_mul_f32 %" #k ", %" #k ", %" #j "\n\t"
            asm volatile(BODY16(I) : P8);
#undef I
        } else if constexpr (K == 2) {
#define I(k, j) "v_pk_add_f32 %" #k ", %" #k ", %" #j "\n\t"
            asm volatile(BODY16(I) : P8);
#undef I
        } else if constexpr (K == 3) {
#define I(k, j) "v_fma_f32 %" #k ", %" #k ", %" #j ", %" #k "\n\t"
            asm volatile(BODY16(I) : R8);
#undef I
        } else if constexpr (K == 4) {
#define I(k, j) "v_pk_fma_f32 %" #k ", %" #k ", %" #j ", %" #k "\n\t"
            asm volatile(BODY16(I) : P8);
#undef I
        } else if constexpr (K == 5) {  // v_cndmask_b32 (no DPP)
#define I(k, j) "v_cndmask_b32 %" #k ", %" #k ", %" #j ", vcc\n\t"
            asm volatile("s_mov_b32 vcc_lo, 0x55555555\n\ts_mov_b32 vcc_hi, 0x55555555\n\t" BODY16(I) : R8 :: "vcc");
#undef I
        } else if constexpr (K == 6) {  // v_cndmask_b32_dpp quad_perm (the xch2 form)
#define I(k, j) "v_cndmask_b32_dpp %" #k ", %" #j ", %" #k ", vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
            asm volatile("s_mov_b32 vcc_lo, 0x55555555\n\ts_mov_b32 vcc_hi, 0x55555555\n\t" BODY16(I) : R8 :: "vcc");
#undef I
        } else if constexpr (K == 7) {  // v_cndmask_b32_dpp row_ror:8
#define I(k, j) "v_cndmask_b32_dpp %" #k ", %" #j ", %" #k ", vcc row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
            asm volatile("s_mov_b32 vcc_lo, 0x55555555\n\ts_mov_b32 vcc_hi, 0x55555555\n\t" BODY16(I) : R8 :: "vcc");
#undef I
        } else if constexpr (K == 8) {  // v_mov_b32_dpp row_ror:8
#define I(k, j) "v_mov_b32_dpp %" #k ", %" #j " row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
            asm volatile(BODY16(I) : R8);
#undef I
        } else if constexpr (K == 9) {  // v_permlane32_swap (pairs k, j)
#define I(k, j) "v_permlane32_swap_b32 %" #k ", %" #j "\n\t"
            asm volatile(BODY16(I) : R8);
#undef I
        } else if constexpr (K == 10) {  // v_permlane16_swap
#define I(k, j) "v_permlane16_swap_b32 %" #k ", %" #j "\n\t"
            asm volatile(BODY16(I) : R8);
#undef I
        } else if constexpr (K == 11) {  // v_add_u32
#define I(k, j) "v_add_u32 %" #k ", %" #k ", %" #j "\n\t"
            asm volatile(BODY16(I) : R8);
#undef I
        } else if constexpr (K == 12) {  // v_perm_b32
#define I(k, j) "v_perm_b32 %" #k ", %" #k ", %" #j ", %" #j "\n\t"
            asm volatile(BODY16(I) : R8);
#undef I
        } else if constexpr (K == 13) {  // ds_read_b32, 16 in flight then wait
#define I(k, j) "ds_read_b32 %" #k ", %8 offset:" #k "\n\t"
            asm volatile(BODY16(I) "s_waitcnt lgkmcnt(0)" : R8 : "v"(t * 4));
#undef I
        } else if constexpr (K == 14) {  // ds_read_b64, 16 in flight then wait
#define I(k, j) "ds_read_b64 %" #k ", %8 offset:" #k "\n\t"
            asm volatile(BODY16(I) "s_waitcnt lgkmcnt(0)" : P8 : "v"(t * 8));
#undef I
        } else if constexpr (K == 15) {  // ds_write_b32
#define I(k, j) "ds_write_b32 %8, %" #k " offset:" #k "\n\t"
            asm volatile(BODY16(I) "s_waitcnt lgkmcnt(0)" : R8 : "v"(t * 4));
#undef I
        } else if constexpr (K == 16) {  // v_pk_mul_f32 with op_sel swap + neg (pk_mul_swap_nlo)
#define I(k, j) "v_pk_mul_f32 %" #k ", %" #k ", %" #j " op_sel:[1,1] op_sel_hi:[0,1] neg_lo:[0,1]\n\t"
            asm volatile(BODY16(I) : P8);
#undef I
        } else if constexpr (K == 17) {  // 1:1 mix v_pk_mul_f32 / v_mul_f32
#define I(k, j) "v_pk_mul_f32 %" #k ", %" #k ", %" #j "\n\tv_mul_f32 %" XS(8) ", %" XS(8) ", %" XS(9) "\n\t"
            asm volatile(I(0, 4) I(1, 5) I(2, 6) I(3, 7) I(4, 0) I(5, 1) I(6, 2) I(7, 3) : P8, "+v"(a[0]), "+v"(a[1]));
#undef I
        } else if constexpr (K == 18) {  // v_mul_f32 dependent chain (latency)
#define I(k, j) "v_mul_f32 %0, %0, %1\n\t"
            asm volatile(BODY16(I) : R8);
#undef I
        } else if constexpr (K == 19) {  // v_pk_mul_f32 dependent chain (latency)
#define I(k, j) "v_pk_mul_f32 %0, %0, %1\n\t"
            asm volatile(BODY16(I) : P8);
#undef I
        } else if constexpr (K == 20) {  // s_nop 0
#define I(k, j) "s_nop 0\n\t"
            asm volatile(BODY16(I) : R8);
#undef I
        } else if constexpr (K == 21) {  // v_cvt_rpi_i32_f32
#define I(k, j) "v_cvt_rpi_i32_f32 %" #k ", %" #j "\n\t"
            asm volatile(BODY16(I) : R8);
#undef I
        } else if constexpr (K == 22) {  // v_cndmask_b32, vcc set once before the loop
#define I(k, j) "v_cndmask_b32 %" #k ", %" #k ", %" #j ", vcc\n\t"
            asm volatile(BODY16(I) : R8 :: "vcc");
#undef I
        } else if constexpr (K == 23) {  // v_cndmask_b32_e64 with an SGPR-pair mask
#define I(k, j) "v_cndmask_b32_e64 %" #k ", %" #k ", %" #j ", %8\n\t"
            asm volatile(BODY16(I) : R8 : "s"(smask));
#undef I
        } else if constexpr (K == 24) {  // v_bfi_b32 with a VGPR lane mask
#define I(k, j) "v_bfi_b32 %" #k ", %8, %" #k ", %" #j "\n\t"
            asm volatile(BODY16(I) : R8 : "v"(vmask));
#undef I
        } else if constexpr (K == 25) {  // v_mov_b32_dpp row_ror:4 bank_mask:0xa (masked write)
#define I(k, j) "v_mov_b32_dpp %" #k ", %" #j " row_ror:4 row_mask:0xf bank_mask:0xa\n\t"
            asm volatile(BODY16(I) : R8);
#undef I
        } else if constexpr (K == 26) {  // v_add_f32_dpp quad_perm
#define I(k, j) "v_add_f32_dpp %" #k ", %" #j ", %" #k " quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
            asm volatile(BODY16(I) : R8);
#undef I
        } else if constexpr (K == 27) {  // v_cndmask_b32 with vcc from a v_cmp before the loop
#define I(k, j) "v_cndmask_b32 %" #k ", %" #k ", %" #j ", vcc\n\t"
            asm volatile("v_cmp_lt_u32 vcc, 31, %0" :: "v"(t & 63) : "vcc");
            asm volatile(BODY16(I) : R8 :: "vcc");
#undef I
        } else if constexpr (K == 28) {  // v_mov_b32_dpp quad_perm (full mask)
#define I(k, j) "v_mov_b32_dpp %" #k ", %" #j " quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
            asm volatile(BODY16(I) : R8);
#undef I
        } else if constexpr (K == 29) {  // v_and_or_b32 select: (a & m) | b
#define I(k, j) "v_and_or_b32 %" #k ", %" #k ", %8, %" #j "\n\t"
            asm volatile(BODY16(I) : R8 : "v"(vmask));
#undef I
        } else if constexpr (K == 30) {  // v_cndmask_b32 where vcc rewritten by s_mov between each pair
#define I(k, j) "v_cndmask_b32 %" #k ", %" #k ", %" #j ", vcc\n\t"
            asm volatile("s_mov_b32 vcc_lo, 0x55555555\n\ts_mov_b32 vcc_hi, 0x55555555\n\t" I(0,4) I(1,5) I(2,6) I(3,7) "s_mov_b32 vcc_lo, 0x33333333\n\ts_mov_b32 vcc_hi, 0x33333333\n\t" I(4,0) I(5,1) I(6,2) I(7,3) "s_mov_b32 vcc_lo, 0x55555555\n\ts_mov_b32 vcc_hi, 0x55555555\n\t" I(0,4) I(1,5) I(2,6) I(3,7) "s_mov_b32 vcc_lo, 0x33333333\n\ts_mov_b32 vcc_hi, 0x33333333\n\t" I(4,0) I(5,1) I(6,2) I(7,3) : R8 :: "vcc");
#undef I
        } else if constexpr (K == 31) {  // v_cndmask_b32_e64 with explicit vcc
#define I(k, j) "v_cndmask_b32_e64 %" #k ", %" #k ", %" #j ", vcc\n\t"
            asm volatile(BODY16(I) : R8 :: "vcc");
#undef I
        } else if constexpr (K == 32) {  // v_add_co_u32_e32 (writes vcc)
#define I(k, j) "v_add_co_u32_e32 %" #k ", vcc, %" #k ", %" #j "\n\t"
            asm volatile(BODY16(I) : R8 :: "vcc");
#undef I
        } else if constexpr (K == 33) {  // v_addc_co_u32_e32 (reads + writes vcc)
#define I(k, j) "v_addc_co_u32_e32 %" #k ", vcc, %" #k ", %" #j ", vcc\n\t"
            asm volatile(BODY16(I) : R8 :: "vcc");
#undef I
        } else if constexpr (K == 34) {  // v_cmp_lt_f32_e32 (writes vcc)
#define I(k, j) "v_cmp_lt_f32_e32 vcc, %" #k ", %" #j "\n\t"
            asm volatile(BODY16(I) : R8 :: "vcc");
#undef I
        } else if constexpr (K == 35) {  // v_cmp_lt_f32_e64 into an SGPR pair
#define I(k, j) "v_cmp_lt_f32_e64 %8, %" #k ", %" #j "\n\t"
            unsigned long long sd;
            asm volatile(BODY16(I) : R8, "=s"(sd));
            (void)sd;
#undef I
        } else if constexpr (K == 36) {  // v_cndmask_b32_e64 with an SGPR pair, in cndmask/dpp pairs
#define I(k, j) "v_mov_b32_dpp %" #k ", %" #j " quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\tv_cndmask_b32_e64 %" #j ", %" #j ", %" #k ", %8\n\t"
            asm volatile(I(0, 4) I(1, 5) I(2, 6) I(3, 7) I(4, 0) I(5, 1) I(6, 2) I(7, 3) : R8 : "s"(smask));
#undef I
        } else if constexpr (K == 37) {  // v_readfirstlane_b32
#define I(k, j) "v_readfirstlane_b32 %8, %" #k "\n\t"
            unsigned sd;
            asm volatile(BODY16(I) : R8, "=s"(sd));
            (void)sd;
#undef I
        } else if constexpr (K == 38) {  // v_lshlrev_b32_sdwa word select
#define I(k, j) "v_lshlrev_b32_sdwa %" #k ", 2, %" #j " dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
            asm volatile(BODY16(I) : R8);
#undef I
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    float s = 0.0f;
#pragma unroll
    for (int i = 0; i < 8; i++) s += a[i] + p[i].x + p[i].y;
    out[blockIdx.x * 256 + t] = s;
    if ((t & 63) == 0) {
        cyc[(blockIdx.x * 4 + (t >> 6)) * 2] = t1 - t0;
        cyc[(blockIdx.x * 4 + (t >> 6)) * 2 + 1] = r1 - r0;
    }
}

static const char* kName[] = {"v_mul_f32",          "v_pk_mul_f32",        "v_pk_add_f32",       "v_fma_f32",
                              "v_pk_fma_f32",       "v_cndmask_b32",       "v_cndmask_dpp quad", "v_cndmask_dpp ror8",
                              "v_mov_b32_dpp ror8", "v_permlane32_swap",   "v_permlane16_swap",  "v_add_u32",
                              "v_perm_b32",         "ds_read_b32",         "ds_read_b64",        "ds_write_b32",
                              "v_pk_mul op_sel/neg", "pk_mul:mul 1:1",     "v_mul chain",        "v_pk_mul chain",
                              "s_nop 0",            "v_cvt_rpi_i32_f32",
                              "v_cndmask vcc once", "v_cndmask_e64 sgpr",  "v_bfi_b32",          "v_mov_dpp ror4 bm",
                              "v_add_f32_dpp quad", "v_cndmask vcc v_cmp", "v_mov_dpp quad",     "v_and_or_b32",
                              "v_cndmask s_mov/4",
                              "v_cndmask_e64 vcc",  "v_add_co_u32_e32",    "v_addc_co_u32_e32",  "v_cmp_lt_f32_e32",
                              "v_cmp_lt_f32_e64 s", "mov_dpp+cndmask_e64", "v_readfirstlane",    "v_lshlrev_sdwa"};

template <int K>
static void run(int waves_per_simd, int iters)
{
    int dev_cus = 0;
    (void)hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = dev_cus * waves_per_simd;  // 256-thread blocks = 1 wave per SIMD each
    float* out;
    unsigned long long* cyc;
    (void)hipMalloc(&out, (size_t)blocks * 256 * 4);
    (void)hipMalloc(&cyc, (size_t)blocks * 4 * 16);
    hipLaunchKernelGGL(rate_kernel<K>, dim3(blocks), dim3(256), 0, 0, out, cyc, iters);
    (void)hipDeviceSynchronize();
    std::vector<unsigned long long> c((size_t)blocks * 8);
    (void)hipMemcpy(c.data(), cyc, c.size() * 8, hipMemcpyDeviceToHost);
    std::vector<double> wc, ghz;
    for (int i = 0; i < blocks * 4; i++) {
        wc.push_back((double)c[2 * i]);
        ghz.push_back((double)c[2 * i] / ((double)c[2 * i + 1] * 10.0));  // memrealtime = 100 MHz
    }
    std::sort(wc.begin(), wc.end());
    std::sort(ghz.begin(), ghz.end());
    const double med = wc[wc.size() / 2];
    const double n_inst = 16.0 * iters;
    printf("%-22s w/SIMD %d: wave %6.2f cyc/inst  SIMD %5.2f cyc/inst  clock %.2f GHz\n", kName[K], waves_per_simd,
           med / n_inst, med / (n_inst * waves_per_simd), ghz[ghz.size() / 2]);
    fflush(stdout);
    (void)hipFree(out);
    (void)hipFree(cyc);
}

template <int K>
static void sweep(int iters)
{
    for (int w : {1, 3, 4, 8}) run<K>(w, iters);
}

template <int... Ks>
static void sweep_all(int iters, std::integer_sequence<int, Ks...>)
{
    (sweep<Ks>(iters), ...);
}

int main(int argc, char** argv)
{
    const int iters = argc > 1 ? atoi(argv[1]) : 2048;
    float* o;
    (void)hipMalloc(&o, 1 << 22);
    hipLaunchKernelGGL(spin_kernel, dim3(4096), dim3(256), 0, 0, o, 100000);
    (void)hipDeviceSynchronize();
    sweep_all(iters, std::make_integer_sequence<int, 39>{});
    return 0;
}
