// clock_probe.hip — does s_memrealtime / s_memtime advance inside a kernel
// (e.g. under rocprofv3 counter collection)?  One wave spins ~N s_sleep
// trips and records both clocks before and after.  Diagnostic tool.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void probe(unsigned long long *out, int trips)
{
    if (threadIdx.x != 0) return;
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime(), t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < trips; ++i) __builtin_amdgcn_s_sleep(8);
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime(), t1 = __builtin_amdgcn_s_memtime();
    out[0] = r0;
    out[1] = r1;
    out[2] = t0;
    out[3] = t1;
}

int main()
{
    unsigned long long *d, h[4];
    if (hipMalloc(&d, 32) != hipSuccess) return 1;
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, 100000);
    if (hipMemcpy(h, d, 32, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    printf("memrealtime delta %llu (100 MHz ticks), memtime delta %llu\n", h[1] - h[0], h[3] - h[2]);
    return 0;
}
