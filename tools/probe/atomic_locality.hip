// Random 4-byte atomicMin / load rates over arrays of growing size: does a
// first[] slice that fits the memory-side cache take atomics much faster than
// the 1.44 GB C5 array?  (DESIGN.md "AnchorFinder at C5")
// build: hipcc -O3 --offload-arch=gfx950 -o tools/probe/atomic_locality tools/probe/atomic_locality.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e = (x);                                                         \
        if (e != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            return 1;                                                               \
        }                                                                           \
    } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

// n random atomicMin over [0, m)
__global__ void k_atomic(uint32_t* a, uint64_t m, int64_t n, uint64_t seed) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t h = mix((uint64_t)i ^ seed);
        atomicMin(&a[h % m], (uint32_t)i);
    }
}

// n random loads over [0, m), summed so they are not dropped
__global__ void k_load(const uint32_t* a, uint64_t m, int64_t n, uint64_t seed, uint32_t* out) {
    uint32_t s = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t h = mix((uint64_t)i ^ seed);
        s += a[h % m];
    }
    if (s == 0x12345678u) out[0] = s;
}

// n random 4-byte / 8-byte plain stores over [0, m) words
__global__ void k_store4(uint32_t* a, uint64_t m, int64_t n, uint64_t seed) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t h = mix((uint64_t)i ^ seed);
        a[h % m] = (uint32_t)i;
    }
}
__global__ void k_store8(uint64_t* a, uint64_t m, int64_t n, uint64_t seed) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t h = mix((uint64_t)i ^ seed);
        a[h % (m / 2)] = (uint64_t)i;
    }
}

int main() {
    const uint64_t sizes_mb[] = {4, 16, 64, 128, 192, 256, 384, 512, 1024, 1472};
    const int64_t n = 256ll << 20;
    uint32_t* a = nullptr;
    uint32_t* out = nullptr;
    CK(hipMalloc(&a, 1472ull << 20));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(a, 0xff, 1472ull << 20));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    printf("array_MB atomic_Gops load_Gops store4_Gops store8_Gops\n");
    for (uint64_t mb : sizes_mb) {
        const uint64_t m = (mb << 20) / 4;
        float ta = 0, tl = 0, t4 = 0, t8 = 0;
        for (int rep = 0; rep < 3; rep++) {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(k_atomic, dim3(8192), dim3(256), 0, 0, a, m, n, (uint64_t)rep * 77);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ta, e0, e1));
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(k_load, dim3(8192), dim3(256), 0, 0, a, m, n, (uint64_t)rep * 91, out);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&tl, e0, e1));
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(k_store4, dim3(8192), dim3(256), 0, 0, a, m, n, (uint64_t)rep * 13);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&t4, e0, e1));
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(k_store8, dim3(8192), dim3(256), 0, 0, (uint64_t*)a, m, n, (uint64_t)rep * 17);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&t8, e0, e1));
        }
        printf("%6llu %8.2f %8.2f %8.2f %8.2f\n", (unsigned long long)mb, n / (ta * 1e6), n / (tl * 1e6),
               n / (t4 * 1e6), n / (t8 * 1e6));
        fflush(stdout);
    }
    return 0;
}
