// FETCH_SIZE calibration for the access widths the fold / outside kernels use
// (MI355X_MICROARCH.md "HBM": only 16-B-per-lane streaming reads are
// calibrated there).  Each kernel reads a 1 GiB buffer once (4x the Infinity
// Cache, so every line comes from HBM) and writes one float per workgroup:
//   dword    one 4-B load per lane, a wave reads 256 contiguous bytes
//            (outside_ring's slot reads, the rings' q5 column loads)
//   dwordx4  one 16-B load per lane (the guide's calibrated case)
//   ubyte    one 1-B load per lane (sequence / code bytes)
// Compare each dispatch's FETCH_SIZE (rocprofv3 --pmc FETCH_SIZE, KB) with
// the 1 GiB it read.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/fetch_calib.hip -o fetch_calib
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr size_t BYTES = size_t(1) << 30;
constexpr int NT = 256;

__global__ void __launch_bounds__(NT) read_dword(const float *__restrict__ a, size_t n, float *out) {
    float s = 0.f;
    for (size_t k = size_t(blockIdx.x) * NT + threadIdx.x; k < n; k += size_t(gridDim.x) * NT) s += a[k];
    if (s == 12345.f) out[blockIdx.x] = s;   // keeps the loads; never true for the zero buffer
}

__global__ void __launch_bounds__(NT) read_dwordx4(const float4 *__restrict__ a, size_t n, float *out) {
    float s = 0.f;
    for (size_t k = size_t(blockIdx.x) * NT + threadIdx.x; k < n; k += size_t(gridDim.x) * NT) {
        const float4 v = a[k];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 12345.f) out[blockIdx.x] = s;
}

__global__ void __launch_bounds__(NT) read_ubyte(const unsigned char *__restrict__ a, size_t n, float *out) {
    unsigned s = 0;
    for (size_t k = size_t(blockIdx.x) * NT + threadIdx.x; k < n; k += size_t(gridDim.x) * NT) s += a[k];
    if (s == 12345u) out[blockIdx.x] = float(s);
}

#define CK(x)                                                              \
    do {                                                                   \
        hipError_t e_ = (x);                                               \
        if (e_ != hipSuccess) {                                            \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));   \
            return 1;                                                      \
        }                                                                  \
    } while (0)

int main() {
    void *buf = nullptr;
    float *out = nullptr;
    CK(hipMalloc(&buf, BYTES));
    CK(hipMalloc(&out, 4096 * sizeof(float)));
    CK(hipMemset(buf, 0, BYTES));
    CK(hipDeviceSynchronize());
    const int grid = 4096;
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(read_dword, dim3(grid), dim3(NT), 0, 0, (const float *)buf, BYTES / 4, out);
        hipLaunchKernelGGL(read_dwordx4, dim3(grid), dim3(NT), 0, 0, (const float4 *)buf, BYTES / 16, out);
        hipLaunchKernelGGL(read_ubyte, dim3(grid), dim3(NT), 0, 0, (const unsigned char *)buf, BYTES, out);
        CK(hipDeviceSynchronize());
    }
    std::printf("each dispatch read %zu bytes (%.0f KB)\n", BYTES, BYTES / 1024.0);
    CK(hipFree(buf));
    CK(hipFree(out));
    return 0;
}
