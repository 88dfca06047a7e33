// Probe: do same-address LDS atomics of one instruction serialise (each lane
// sees the others' earlier effects) on this GPU?  Prints, for 64 lanes doing
// atomicOr(&w, bit) on one word: how many lanes saw the bit already set, and
// for atomicAdd(&w, 1): the distinct return values.
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(unsigned* out)
{
    __shared__ unsigned w[4];
    const unsigned l = threadIdx.x;
    if (l < 4) w[l] = 0;
    __syncthreads();
    unsigned o = atomicOr(&w[0], 1u);                 // same bit, same word
    unsigned o2 = atomicOr(&w[1], 1u << (l & 31));    // different bits, same word
    unsigned a = atomicAdd(&w[2], 1u);
    out[l] = o;
    out[64 + l] = o2;
    out[128 + l] = a;
}
int main()
{
    unsigned* d; unsigned h[192];
    hipMalloc(&d, sizeof(h));
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    int seen = 0, seen2 = 0;
    for (int i = 0; i < 64; i++) { seen += (h[i] & 1) != 0; seen2 += (h[64 + i] & (1u << (i & 31))) != 0; }
    printf("same bit: %d of 64 lanes saw it set (serialised: 63)\n", seen);
    printf("own bit seen set (lanes 32-63 share bits with 0-31): %d\n", seen2);
    printf("atomicAdd returns:");
    for (int i = 0; i < 64; i++) printf(" %u", h[128 + i]);
    printf("\n");
    return 0;
}
