// Workgroups per CU the runtime admits for a 256-thread kernel at a given dynamic LDS size
// (which LDS footprints keep 3 workgroups = 3 waves/SIMD per CU).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void __launch_bounds__(256, 1) k(int* o) {
    extern __shared__ int lds[];
    lds[threadIdx.x] = threadIdx.x;
    __syncthreads();
    o[threadIdx.x] = lds[255 - threadIdx.x];
}
int main() {
    hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    for (int bytes : {35392, 40960, 49728, 53248, 53760, 53824, 54272, 54613, 55296}) {
        int n = 0;
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, 256, bytes);
        printf("dynamic LDS %6d B -> %d workgroups/CU\n", bytes, n);
    }
    return 0;
}
