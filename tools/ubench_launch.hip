// Microbenchmark: the fixed cost of a kernel boundary on MI355X, to decide
// between more fused launches and a cooperative (grid-barrier) pass chain.
//   1. back-to-back empty kernels of the eval / pass grid shapes (hipEvents
//      around 200 launches on one stream);
//   2. a VALU-busy kernel (~10 us) run as 1 launch of 2x work vs 2 launches
//      of 1x work: the difference is the boundary cost between two full-chip
//      kernels (drain + dispatch);
//   3. a cooperative kernel of the pass grid shape doing K grid barriers
//      (cooperative_groups grid.sync): the cost of one barrier.
#include <hip/hip_runtime.h>
#include <hip/hip_cooperative_groups.h>
#include <cstdio>
namespace cg = cooperative_groups;

__global__ void empty_k(unsigned* out) {
    if (out && blockIdx.x == 0xFFFFFFFFu) out[0] = 1;
}
__global__ void __launch_bounds__(256) busy_k(unsigned* out, int iters) {
    unsigned v0 = threadIdx.x, v1 = v0 * 3u, v2 = v0 * 5u, v3 = v0 * 7u;
    for (int i = 0; i < iters; i++) {
        v0 = __builtin_amdgcn_perm(v1, v0, 0x03020100u + i);
        v1 = __builtin_amdgcn_perm(v2, v1, 0x01000302u + i);
        v2 = __builtin_amdgcn_perm(v3, v2, 0x02010003u + i);
        v3 = __builtin_amdgcn_perm(v0, v3, 0x00030201u + i);
    }
    if ((v0 ^ v1 ^ v2 ^ v3) == 0x12345678u) out[blockIdx.x] = 1;
}
__global__ void __launch_bounds__(256) coop_k(unsigned* out, int syncs) {
    cg::grid_group g = cg::this_grid();
    for (int i = 0; i < syncs; i++) g.sync();
    if (out && threadIdx.x == 0 && blockIdx.x == 0) out[0] = syncs;
}

static float elapsed(hipEvent_t a, hipEvent_t b) {
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main() {
    unsigned* d;
    hipMalloc(&d, 1 << 20);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int N = 200;
    struct { int g, t; } shapes[] = {{256, 64}, {256, 256}, {1024, 256}, {512, 512}};
    for (auto s : shapes) {
        for (int i = 0; i < 10; i++) empty_k<<<s.g, s.t>>>(d);
        hipEventRecord(a);
        for (int i = 0; i < N; i++) empty_k<<<s.g, s.t>>>(d);
        hipEventRecord(b);
        printf("empty kernel %5d x %3d: %.2f us per launch (back to back)\n", s.g, s.t, elapsed(a, b) * 1e3 / N);
    }
    for (int iters : {2000, 4000}) {
        busy_k<<<1024, 256>>>(d, iters);
        hipEventRecord(a);
        for (int i = 0; i < 20; i++) busy_k<<<1024, 256>>>(d, iters);
        hipEventRecord(b);
        const float one = elapsed(a, b) * 1e3 / 20;
        hipEventRecord(a);
        for (int i = 0; i < 20; i++) {
            busy_k<<<1024, 256>>>(d, iters / 2);
            busy_k<<<1024, 256>>>(d, iters / 2);
        }
        hipEventRecord(b);
        const float two = elapsed(a, b) * 1e3 / 20;
        printf("busy 1024 x 256, %d iters: 1 launch %.2f us, 2 half launches %.2f us -> boundary %.2f us\n", iters, one,
               two, two - one);
    }
    int dev = 0, coop = 0;
    hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev);
    printf("cooperative launch supported: %d\n", coop);
    if (coop) {
        for (int grid : {256, 1024}) {
            for (int syncs : {0, 100}) {
                int sy = syncs;
                unsigned* dp = d;
                void* args[] = {&dp, &sy};
                hipError_t e = hipLaunchCooperativeKernel((const void*)coop_k, dim3(grid), dim3(256), args, 0, 0);
                hipEventRecord(a);
                for (int r = 0; r < 5 && e == hipSuccess; r++)
                    e = hipLaunchCooperativeKernel((const void*)coop_k, dim3(grid), dim3(256), args, 0, 0);
                hipEventRecord(b);
                const float ms = elapsed(a, b);
                printf("cooperative %4d x 256, %3d grid syncs: %s %.2f us per launch\n", grid, syncs,
                       e == hipSuccess ? "ok" : hipGetErrorString(e), ms * 1e3 / 5);
            }
        }
    }
    hipError_t e = hipDeviceSynchronize();
    printf("done: %s\n", hipGetErrorString(e));
    return 0;
}
