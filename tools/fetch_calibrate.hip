// fetch_calibrate.hip — what rocprofv3's FETCH_SIZE / TCC_EA0_RDREQ* report
// on gfx950 for the access shapes of the render's trace kernel, on a KNOWN
// number of touched 128-B lines (MI355X_MICROARCH.md, HBM section: "calibrate
// on a known byte count in your own access pattern before trusting an
// absolute").
//
// Buffer: 4 GiB (16x the 256 MiB Infinity Cache), so every touched line comes
// from HBM.  Each dispatch touches every line of a 1 GiB window exactly once
// (line = i * odd constant mod 2^23, a bijection; windows evicted between uses):
//   stream16 : 16 B per lane, contiguous (the guide's known x2 case)
//   gather8  : one 8-B load at a random line (KD node fetch shape)
//   gather16 : one 16-B load at a random line (plane stream shape)
//   gather64 : 3 x 16 B + 8 B of one 64-B record at a random line (barycentric
//              record shape)
//   gather128: 8 x 16 B covering one whole random line
// Build: hipcc --offload-arch=gfx950 -O3 tools/fetch_calibrate.hip -o /tmp/fetch_calibrate
// Run under: rocprofv3 --pmc FETCH_SIZE --kernel-trace -- /tmp/fetch_calibrate
// Prints the dispatch order and the lines each dispatch touches.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <numeric>
#include <random>
#include <vector>

#define CHK(x)                                                                                   \
    do {                                                                                         \
        hipError_t e_ = (x);                                                                     \
        if (e_ != hipSuccess) {                                                                  \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                              \
            exit(1);                                                                             \
        }                                                                                        \
    } while (0)

static const size_t WINDOW = 1ull << 30; // bytes per dispatch
static const size_t LINES = WINDOW / 128;

__global__ void stream16(const uint4 *__restrict__ p, size_t n16, unsigned *sink)
{
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9e3779b9u) atomicAdd(sink, 1u);
}

// line of thread i: i * odd constant mod 2^23 — a bijection on the window's
// lines, so each is touched exactly once, with no permutation array to read
template <int SHAPE>
__global__ void gather(const uint8_t *__restrict__ base, size_t n, unsigned *sink)
{
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint8_t *line = base + (size_t)(((uint32_t)i * 0x9E3779B1u) & (uint32_t)(n - 1)) * 128;
        if (SHAPE == 8) {
            const uint2 v = *reinterpret_cast<const uint2 *>(line);
            acc ^= v.x ^ v.y;
        } else if (SHAPE == 16) {
            const uint4 v = *reinterpret_cast<const uint4 *>(line);
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        } else if (SHAPE == 64) {
            const uint4 a = reinterpret_cast<const uint4 *>(line)[0], b = reinterpret_cast<const uint4 *>(line)[1],
                        c = reinterpret_cast<const uint4 *>(line)[2];
            const uint2 d = reinterpret_cast<const uint2 *>(line)[6];
            acc ^= a.x ^ b.y ^ c.z ^ d.x ^ a.w ^ b.w ^ c.w ^ d.y;
        } else {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const uint4 v = reinterpret_cast<const uint4 *>(line)[k];
                acc ^= v.x ^ v.y ^ v.z ^ v.w;
            }
        }
    }
    if (acc == 0x9e3779b9u) atomicAdd(sink, 1u);
}

__global__ void fill(uint4 *p, size_t n16)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
        p[i] = make_uint4((uint32_t)i, (uint32_t)(i >> 32) ^ 0x55u, 7u, (uint32_t)i * 2654435761u);
}

__global__ void marker() {}

int main()
{
    const size_t windows = 4;
    uint8_t *buf = nullptr;
    unsigned *sink = nullptr;
    CHK(hipMalloc(&buf, windows * WINDOW));
    CHK(hipMalloc(&sink, 4));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, (uint4 *)buf, windows * WINDOW / 16);
    CHK(hipDeviceSynchronize());
    // flush the Infinity Cache of the fill: stream another window's worth first
    hipLaunchKernelGGL(stream16, dim3(8192), dim3(256), 0, 0, (const uint4 *)(buf + 3 * WINDOW), WINDOW / 16, sink);
    CHK(hipDeviceSynchronize());
    printf("{\"lines_per_dispatch\": %zu, \"window_bytes\": %zu, \"order\": [", LINES, WINDOW);
    const char *names[] = {"stream16", "gather8", "gather16", "gather64", "gather128"};
    for (int k = 0; k < 5; ++k) {
        const uint8_t *w = buf + (size_t)(k % 3) * WINDOW; // window 0,1,2,0,1: each re-read window was evicted
        hipLaunchKernelGGL(marker, dim3(1), dim3(64), 0, 0);
        switch (k) {
        case 0: hipLaunchKernelGGL(stream16, dim3(8192), dim3(256), 0, 0, (const uint4 *)w, WINDOW / 16, sink); break;
        case 1: hipLaunchKernelGGL(gather<8>, dim3(8192), dim3(256), 0, 0, w, LINES, sink); break;
        case 2: hipLaunchKernelGGL(gather<16>, dim3(8192), dim3(256), 0, 0, w, LINES, sink); break;
        case 3: hipLaunchKernelGGL(gather<64>, dim3(8192), dim3(256), 0, 0, w, LINES, sink); break;
        default: hipLaunchKernelGGL(gather<128>, dim3(8192), dim3(256), 0, 0, w, LINES, sink); break;
        }
        CHK(hipDeviceSynchronize());
        printf("%s\"%s\"", k ? ", " : "", names[k]);
    }
    printf("]}\n");
    CHK(hipFree(buf));
    CHK(hipFree(sink));
    return 0;
}
