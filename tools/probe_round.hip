// Probe: does v_cvt_rpi_i32_f32 (+ v_cvt_pk_i16_i32 saturation) reproduce Java's
// Math.round(float) followed by SampleBuffer's short clamp, for EVERY float bit pattern?
// Reference formula (exact): y = floor(x); r = (x - y >= 0.5) ? y + 1 : y; cvt_i32 (NaN -> 0,
// saturating); clamp to [-32768, 32767].
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ int ref_round16(float x)
{
    float y = __builtin_floorf(x);
    float r = (x - y >= 0.5f) ? y + 1.0f : y;
    int v;
    asm volatile("v_cvt_i32_f32 %0, %1" : "=v"(v) : "v"(r));
    return v < -32768 ? -32768 : (v > 32767 ? 32767 : v);
}

__global__ void probe(uint32_t base, unsigned long long* bad, uint32_t* first)
{
    uint32_t bits = base + blockIdx.x * blockDim.x + threadIdx.x;
    float x = __uint_as_float(bits);
    uint32_t w;
    int a;
    asm volatile("v_cvt_rpi_i32_f32 %0, %1" : "=v"(a) : "v"(x));
    asm volatile("v_cvt_pk_i16_i32 %0, %1, %2" : "=v"(w) : "v"(a), "v"(a));
    int got = (int16_t)(w & 0xffff);
    int got_hi = (int16_t)(w >> 16);
    int want = ref_round16(x);
    if (got != want || got_hi != want) {
        atomicAdd(bad, 1ull);
        atomicMin(first, bits);
    }
}

int main()
{
    unsigned long long* bad;
    uint32_t* first;
    hipMalloc(&bad, 8);
    hipMalloc(&first, 4);
    hipMemset(bad, 0, 8);
    hipMemset(first, 0xff, 4);
    const uint32_t chunk = 1u << 28;
    for (uint64_t b = 0; b < (1ull << 32); b += chunk)
        hipLaunchKernelGGL(probe, dim3(chunk / 256), dim3(256), 0, 0, (uint32_t)b, bad, first);
    unsigned long long hb;
    uint32_t hf;
    hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost);
    hipMemcpy(&hf, first, 4, hipMemcpyDeviceToHost);
    printf("mismatches over all 2^32 floats: %llu (first bits 0x%08x = %g)\n", hb, hf, (double)__builtin_bit_cast(float, hf));
    return hb != 0;
}
