// FETCH_SIZE calibration for the access patterns of the pre-order kernels (MI355X guide, HBM:
// "other access widths are uncalibrated: calibrate on a known byte count in your own access
// pattern").  Each kernel reads a known set of 16-B words out of a 4 GiB buffer (far past the
// 256 MiB Infinity Cache) and folds them into one vector store per lane:
//   stream      every 16-B word, lanes contiguous (the guide's calibrated case)
//   s128        one 16-B word per 128-B line (lane t: word 8t)
//   s64         one 16-B word per 64-B sector (lane t: word 4t), both sectors of each line
//   s64x2       one 16-B word per other 64-B sector (lane t: word 8t + 4): one sector per line
//   row64       64 contiguous bytes per lane, one lane per 128-B line (k_tail's sub_planes rows)
//   rand        one 16-B word at a hashed position per lane (scattered parent finals)
// Build: hipcc -O3 --offload-arch=gfx950 tools/calib_fetch.hip -o /tmp/calib_fetch
// Run:   rocprofv3 --pmc FETCH_SIZE ... -- /tmp/calib_fetch   (one pass per counter set)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__global__ void k_fill(uint4* b, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        b[i] = make_uint4((uint32_t)i, (uint32_t)(i >> 32), 7u, 9u);
}

__device__ __forceinline__ void sink(uint4* out, uint4 a) { out[blockIdx.x * (size_t)blockDim.x + threadIdx.x] = a; }

__device__ __forceinline__ void acc(uint4& a, const uint4& v) { a.x ^= v.x; a.y ^= v.y; a.z ^= v.z; a.w ^= v.w; }

__global__ void k_stream(const uint4* b, size_t n, uint4* out) {
    uint4 a = make_uint4(0, 0, 0, 0);
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) acc(a, b[i]);
    sink(out, a);
}

// lane t (over the whole grid, grid-stride) reads word t * stride + off
__global__ void k_stride(const uint4* b, size_t n, int stride, int off, uint4* out) {
    uint4 a = make_uint4(0, 0, 0, 0);
    for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t * stride + off < n; t += (size_t)gridDim.x * blockDim.x)
        acc(a, b[t * stride + off]);
    sink(out, a);
}

__global__ void k_row64(const uint4* b, size_t n, uint4* out) {
    uint4 a = make_uint4(0, 0, 0, 0);
    for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t * 8 + 3 < n; t += (size_t)gridDim.x * blockDim.x) {
        const uint4* p = b + t * 8;
        acc(a, p[0]); acc(a, p[1]); acc(a, p[2]); acc(a, p[3]);
    }
    sink(out, a);
}

__global__ void k_rand(const uint4* b, size_t n, size_t reads, uint4* out) {
    uint4 a = make_uint4(0, 0, 0, 0);
    for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < reads; t += (size_t)gridDim.x * blockDim.x) {
        uint64_t h = (t + 1) * 0x9E3779B97F4A7C15ull;
        h ^= h >> 29;
        h *= 0xBF58476D1CE4E5B9ull;
        h ^= h >> 32;
        acc(a, b[h % n]);
    }
    sink(out, a);
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
    const size_t bytes = 4ull << 30, n = bytes / 16;
    const int grid = 256 * 64, block = 256;   // 16384 workgroups x 4 waves, grid-stride
    uint4 *b = nullptr, *out = nullptr;
    CK(hipMalloc(&b, bytes));
    CK(hipMalloc(&out, (size_t)grid * block * sizeof(uint4)));
    hipLaunchKernelGGL(k_fill, dim3(grid), dim3(block), 0, 0, b, n);
    CK(hipDeviceSynchronize());
    const size_t rand_reads = n / 8;   // as many reads as s128 has lines
    // (name, useful bytes, 64-B sectors, 128-B lines touched)
    std::printf("kernel useful_bytes sectors64 lines128\n");
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k_stream, dim3(grid), dim3(block), 0, 0, b, n, out);
        hipLaunchKernelGGL(k_stride, dim3(grid), dim3(block), 0, 0, b, n, 8, 0, out);
        hipLaunchKernelGGL(k_stride, dim3(grid), dim3(block), 0, 0, b, n, 4, 0, out);
        hipLaunchKernelGGL(k_stride, dim3(grid), dim3(block), 0, 0, b, n, 8, 4, out);
        hipLaunchKernelGGL(k_row64, dim3(grid), dim3(block), 0, 0, b, n, out);
        hipLaunchKernelGGL(k_rand, dim3(grid), dim3(block), 0, 0, b, n, rand_reads, out);
        CK(hipDeviceSynchronize());
    }
    std::printf("stream %zu %zu %zu\n", bytes, bytes / 64, bytes / 128);
    std::printf("stride8 (s128) %zu %zu %zu\n", n / 8 * 16, n / 8, n / 8);
    std::printf("stride4 (s64) %zu %zu %zu\n", n / 4 * 16, n / 4, n / 8);
    std::printf("stride8+4 (s64x2) %zu %zu %zu\n", n / 8 * 16, n / 8, n / 8);
    std::printf("row64 %zu %zu %zu\n", n / 8 * 64, n / 8, n / 8);
    std::printf("rand %zu ~%zu ~%zu\n", rand_reads * 16, rand_reads, rand_reads);
    CK(hipFree(b));
    CK(hipFree(out));
    return 0;
}
