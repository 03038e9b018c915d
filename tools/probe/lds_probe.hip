// Probe: LDS limits per workgroup on this device (diagnostic only).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int n, int* out) {
    extern __shared__ int s[];
    for (int i = threadIdx.x; i < n; i += blockDim.x) s[i] = i;
    __syncthreads();
    if (threadIdx.x == 0) out[0] = s[n - 1];
}
int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    printf("sharedMemPerBlock %zu maxSharedMemoryPerMultiProcessor %zu sharedMemPerBlockOptin %zu\n",
           p.sharedMemPerBlock, p.maxSharedMemoryPerMultiProcessor, p.sharedMemPerBlockOptin);
    int* d;
    hipMalloc(&d, 4);
    for (int kb : {64, 96, 128, 160}) {
        size_t bytes = (size_t)kb * 1024;
        hipError_t e0 = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
        hipLaunchKernelGGL(k, dim3(1), dim3(64), bytes, 0, (int)(bytes / 4), d);
        hipError_t e1 = hipGetLastError();
        hipError_t e2 = hipDeviceSynchronize();
        int h = -1;
        hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
        printf("%d KB: attr %s launch %s sync %s out %d\n", kb, hipGetErrorString(e0), hipGetErrorString(e1),
               hipGetErrorString(e2), h);
    }
    return 0;
}
