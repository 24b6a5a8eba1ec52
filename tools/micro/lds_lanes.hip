// Microbenchmark: LDS time of ds_read_b32 against the number of active lanes.
// Each wave issues R rounds of 16 reads with `active` lanes enabled; prints ms per
// variant.  Note the addresses: lane stride 8 words puts every 4th lane on one
// bank, so this measures a bank-conflicted pattern (time ~ active lanes); a
// conflict-free read costs one LDS cycle per 32-lane group whatever the lanes.
// (diagnostic, not product code)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__global__ void __launch_bounds__(512) k(uint32_t *out, int rounds, int active) {
    __shared__ uint32_t sm[16384];
    for (int t = threadIdx.x; t < 16384; t += 512) sm[t] = t * 2654435761u;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    uint32_t acc = 0;
    if (lane < active) {
        uint32_t base = (threadIdx.x * 7) & 8191;
        for (int r = 0; r < rounds; r++) {
            uint32_t v[16];
#pragma unroll
            for (int k = 0; k < 16; k++) v[k] = sm[(base + k * 64 + lane) & 16383];
#pragma unroll
            for (int k = 0; k < 16; k++) acc += v[k];
            base = (base + acc) & 8191;
        }
    }
    out[blockIdx.x * 512 + threadIdx.x] = acc;
}
int main() {
    uint32_t *d;
    hipMalloc(&d, 512 * 4096 * 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int act : {64, 48, 33, 32, 20, 16, 1}) {
        for (int rep = 0; rep < 2; rep++) {
            hipEventRecord(a);
            hipLaunchKernelGGL(k, dim3(2048), dim3(512), 0, 0, d, 2000, act);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            if (rep) printf("active lanes %2d: %.3f ms\n", act, ms);
        }
    }
    return 0;
}
