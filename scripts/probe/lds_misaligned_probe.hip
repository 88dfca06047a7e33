// Probe: are misaligned ds_read_b128 / ds_write_b128 / b64 / b32 / b16 exact
// on this GPU (SH_MEM_CONFIG unaligned mode), and what do they cost?
// Prints mismatch counts per width and misalignment, and cycles per wave
// instruction for aligned against misaligned b128 reads and writes.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint32_t v2u __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint4 rd128(uint32_t a)
{
    v4u v;
    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void wr128(uint32_t a, uint4 v)
{
    v4u t = {v.x, v.y, v.z, v.w};
    asm volatile("ds_write_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : : "v"(a), "v"(t) : "memory");
}
__device__ __forceinline__ void wr64(uint32_t a, uint2 v)
{
    v2u t = {v.x, v.y};
    asm volatile("ds_write_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : : "v"(a), "v"(t) : "memory");
}
__device__ __forceinline__ void wr32(uint32_t a, uint32_t v)
{
    asm volatile("ds_write_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : : "v"(a), "v"(v) : "memory");
}
__device__ __forceinline__ void wr16(uint32_t a, uint32_t v)
{
    asm volatile("ds_write_b16 %0, %1\n\ts_waitcnt lgkmcnt(0)" : : "v"(a), "v"(v) : "memory");
}

__global__ void k(uint32_t* out, uint32_t mis, uint64_t* cyc)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[8192];
    const uint32_t l = threadIdx.x;
    const uint32_t base = (uint32_t)(uintptr_t)lds;
    for (uint32_t i = l; i < 8192; i += 64)
        lds[i] = (uint8_t)(i * 7 + 3);
    __syncthreads();
    // reads: lane l reads 16 bytes at 32*l + mis
    const uint32_t a = 32 * l + mis;
    uint4 v = rd128(base + a);
    uint32_t bad = 0;
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    for (int i = 0; i < 16; i++)
        bad += ((w[i / 4] >> (8 * (i % 4))) & 0xFF) != (uint8_t)((a + i) * 7 + 3);
    // writes: lane l writes 16 bytes at 4096 + 32*l + mis, pattern from its id
    const uint32_t wa = 4096 + 32 * l + mis;
    wr128(base + wa, make_uint4(0x03020100u + l, 0x07060504u + l, 0x0B0A0908u + l, 0x0F0E0D0Cu + l));
    __syncthreads();
    uint32_t badw = 0;
    for (int i = 0; i < 16; i++) {
        const uint32_t word = i < 4 ? 0x03020100u + l : i < 8 ? 0x07060504u + l : i < 12 ? 0x0B0A0908u + l : 0x0F0E0D0Cu + l;
        badw += lds[wa + i] != (uint8_t)(word >> (8 * (i % 4)));
    }
    // neighbours untouched
    badw += lds[wa - 1] != (uint8_t)((wa - 1) * 7 + 3);
    badw += lds[wa + 16] != (uint8_t)((wa + 16) * 7 + 3);
    __syncthreads();
    // b64 / b32 / b16 at 4096 + 32*l + 16 + mis (inside this lane's 32 bytes: mis <= 7)
    const uint32_t sa = 4096 + 32 * l + 16 + (mis & 7);
    wr64(base + sa, make_uint2(0xA1A2A3A4u, 0xB1B2B3B4u));
    __syncthreads();
    uint32_t bad64 = 0;
    for (int i = 0; i < 8; i++)
        bad64 += lds[sa + i] != (uint8_t)((i < 4 ? 0xA1A2A3A4u : 0xB1B2B3B4u) >> (8 * (i % 4)));
    wr32(base + sa, 0xC1C2C3C4u);
    wr16(base + sa + 4, 0xD1D2u);
    __syncthreads();
    uint32_t bad32 = 0;
    for (int i = 0; i < 4; i++)
        bad32 += lds[sa + i] != (uint8_t)(0xC1C2C3C4u >> (8 * i));
    bad32 += lds[sa + 4] != 0xD2 || lds[sa + 5] != 0xD1 || lds[sa + 6] != 0xB2;
    out[l] = bad;
    out[64 + l] = badw;
    out[128 + l] = bad64;
    out[192 + l] = bad32;
    // timing: 256 dependent-free b128 reads at this misalignment
    __syncthreads();
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    uint32_t acc = 0;
#pragma unroll 1
    for (int r = 0; r < 256; r++) {
        uint4 t = rd128(base + ((a + 48 * r) & 4095));
        acc += t.x;
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int r = 0; r < 256; r++)
        wr128(base + 4096 + ((a + 48 * r) & 4079), make_uint4(acc, r, l, 0));
    uint64_t t2 = __builtin_amdgcn_s_memtime();
    if (l == 0) {
        cyc[0] = t1 - t0;
        cyc[1] = t2 - t1;
    }
    out[256 + l] = acc;
}

int main()
{
    uint32_t* d;
    uint64_t* dc;
    uint32_t h[320];
    uint64_t c[2];
    if (hipMalloc(&d, sizeof(h)) || hipMalloc(&dc, sizeof(c))) return 1;
    int fails = 0;
    for (uint32_t mis = 0; mis < 16; mis++) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, mis, dc);
        if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) ||
            hipMemcpy(c, dc, sizeof(c), hipMemcpyDeviceToHost))
            return 1;
        uint32_t s[4] = {0, 0, 0, 0};
        for (int i = 0; i < 64; i++)
            for (int j = 0; j < 4; j++)
                s[j] += h[64 * j + i];
        printf("mis %2u: bad bytes read128 %u write128 %u write64 %u write32/16 %u | "
               "memtime/256 reads %llu, /256 writes %llu\n",
               mis, s[0], s[1], s[2], s[3], (unsigned long long)c[0], (unsigned long long)c[1]);
        fails += s[0] + s[1] + s[2] + s[3];
    }
    printf(fails ? "MISALIGNED LDS: NOT EXACT\n" : "MISALIGNED LDS: exact\n");
    return 0;
}
