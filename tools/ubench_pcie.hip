// Host-link copies by kernel versus by the copy engines (diagnostic, not
// product code).  Pinned host buffers (hipHostMalloc) are device-accessible,
// so a kernel can move stripe rows over the link itself: this measures
//   - hipMemcpyAsync H2D, D2H, and both at once on two streams,
//   - a copy kernel H2D (reads host, writes HBM), D2H (reads HBM, writes host),
//   - one kernel doing both directions at once (half its workgroups each way),
// 32 MiB per direction, best of 5 after 3 warm-ups, GB/s per direction.
// Build: hipcc -O3 --offload-arch=gfx950 tools/ubench_pcie.hip -o /tmp/ubench_pcie
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// blocks [0, split) copy a -> b, blocks [split, grid) copy c -> d; n16 16-byte words each
__global__ void __launch_bounds__(256) copy2(const u32x4* a, u32x4* b, const u32x4* c, u32x4* d, size_t n16,
                                             unsigned split) {
    const bool first = blockIdx.x < split;
    const unsigned nb = first ? split : gridDim.x - split;
    const unsigned bi = first ? blockIdx.x : blockIdx.x - split;
    const u32x4* src = first ? a : c;
    u32x4* dst = first ? b : d;
    const size_t stride = (size_t)nb * 256 * 4;
    for (size_t i = (size_t)bi * 256 * 4 + threadIdx.x; i < n16; i += stride) {
        u32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) v[u] = i + u * 256 < n16 ? src[i + u * 256] : u32x4{0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < 4; u++)
            if (i + u * 256 < n16) dst[i + u * 256] = v[u];
    }
}

int main(int argc, char** argv) {
    const size_t bytes = (size_t)32 << 20, n16 = bytes / 16;
    const unsigned blocks = argc > 1 ? atoi(argv[1]) : 256;
    void *h_in, *h_out, *d_a, *d_b;
    CK(hipHostMalloc(&h_in, bytes, hipHostMallocDefault));
    CK(hipHostMalloc(&h_out, bytes, hipHostMallocDefault));
    CK(hipMalloc(&d_a, bytes));
    CK(hipMalloc(&d_b, bytes));
    memset(h_in, 1, bytes);
    memset(h_out, 2, bytes);
    {
        // where this process runs and where its pinned pages live (NUMA node of
        // the first page of each buffer, move_pages with no target = query)
        void* pages[2] = {h_in, h_out};
        int status[2] = {-1, -1};
        const long rc = syscall(SYS_move_pages, 0, 2, pages, nullptr, status, 0);
        printf("cpu %d, pinned pages on NUMA nodes %d / %d (move_pages rc %ld)\n", sched_getcpu(), status[0], status[1], rc);
    }
    CK(hipMemset(d_a, 3, bytes));
    CK(hipMemset(d_b, 4, bytes));
    hipStream_t s0, s1;
    CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto time = [&](const char* name, int dirs, auto body) {
        float best = 1e9f;
        for (int r = 0; r < 8; r++) {
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, s0));
            body();
            CK(hipEventRecord(e1, s0));
            CK(hipEventSynchronize(e1));
            CK(hipDeviceSynchronize());
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 3 && ms < best) best = ms;
        }
        printf("%-34s %8.3f ms  %6.1f GB/s per direction (%d dir)\n", name, best, bytes / (best * 1e6), dirs);
    };
    time("memcpy H2D", 1, [&] { CK(hipMemcpyAsync(d_a, h_in, bytes, hipMemcpyHostToDevice, s0)); });
    time("memcpy D2H", 1, [&] { CK(hipMemcpyAsync(h_out, d_b, bytes, hipMemcpyDeviceToHost, s0)); });
    time("memcpy H2D + D2H on two streams", 2, [&] {
        hipEvent_t f;
        CK(hipEventCreateWithFlags(&f, hipEventDisableTiming));
        CK(hipEventRecord(f, s0));
        CK(hipStreamWaitEvent(s1, f, 0));
        CK(hipEventDestroy(f));
        CK(hipMemcpyAsync(d_a, h_in, bytes, hipMemcpyHostToDevice, s0));
        CK(hipMemcpyAsync(h_out, d_b, bytes, hipMemcpyDeviceToHost, s1));
        hipEvent_t j;
        CK(hipEventCreateWithFlags(&j, hipEventDisableTiming));
        CK(hipEventRecord(j, s1));
        CK(hipStreamWaitEvent(s0, j, 0));
        CK(hipEventDestroy(j));
    });
    time("kernel H2D", 1, [&] {
        hipLaunchKernelGGL(copy2, dim3(blocks), dim3(256), 0, s0, (const u32x4*)h_in, (u32x4*)d_a,
                           (const u32x4*)h_in, (u32x4*)d_a, n16, blocks);
    });
    time("kernel D2H", 1, [&] {
        hipLaunchKernelGGL(copy2, dim3(blocks), dim3(256), 0, s0, (const u32x4*)d_b, (u32x4*)h_out,
                           (const u32x4*)d_b, (u32x4*)h_out, n16, blocks);
    });
    time("kernel H2D + D2H in one launch", 2, [&] {
        hipLaunchKernelGGL(copy2, dim3(2 * blocks), dim3(256), 0, s0, (const u32x4*)h_in, (u32x4*)d_a,
                           (const u32x4*)d_b, (u32x4*)h_out, n16, blocks);
    });
    // a copy engine one way, a copy kernel the other way (no two copy-engine
    // jobs that could be queued on one engine)
    time("memcpy H2D + kernel D2H", 2, [&] {
        hipEvent_t f;
        CK(hipEventCreateWithFlags(&f, hipEventDisableTiming));
        CK(hipEventRecord(f, s0));
        CK(hipStreamWaitEvent(s1, f, 0));
        CK(hipEventDestroy(f));
        CK(hipMemcpyAsync(d_a, h_in, bytes, hipMemcpyHostToDevice, s0));
        hipLaunchKernelGGL(copy2, dim3(blocks), dim3(256), 0, s1, (const u32x4*)d_b, (u32x4*)h_out,
                           (const u32x4*)d_b, (u32x4*)h_out, n16, blocks);
        hipEvent_t j;
        CK(hipEventCreateWithFlags(&j, hipEventDisableTiming));
        CK(hipEventRecord(j, s1));
        CK(hipStreamWaitEvent(s0, j, 0));
        CK(hipEventDestroy(j));
    });
    // H2D on stream a, D2H on stream b, for pairs of 4 streams: which pairs
    // overlap (copy engines per stream are the runtime's choice)
    hipStream_t ss[4];
    for (auto& x : ss) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
    for (int a = 0; a < 4; a++)
        for (int b = 0; b < 4; b++) {
            if (a == b) continue;
            char name[64];
            snprintf(name, sizeof name, "memcpy H2D s%d + D2H s%d", a, b);
            time(name, 2, [&] {
                hipEvent_t f;
                CK(hipEventCreateWithFlags(&f, hipEventDisableTiming));
                CK(hipEventRecord(f, s0));
                CK(hipStreamWaitEvent(ss[a], f, 0));
                CK(hipStreamWaitEvent(ss[b], f, 0));
                CK(hipEventDestroy(f));
                CK(hipMemcpyAsync(d_a, h_in, bytes, hipMemcpyHostToDevice, ss[a]));
                CK(hipMemcpyAsync(h_out, d_b, bytes, hipMemcpyDeviceToHost, ss[b]));
                hipEvent_t j0, j1;
                CK(hipEventCreateWithFlags(&j0, hipEventDisableTiming));
                CK(hipEventCreateWithFlags(&j1, hipEventDisableTiming));
                CK(hipEventRecord(j0, ss[a]));
                CK(hipEventRecord(j1, ss[b]));
                CK(hipStreamWaitEvent(s0, j0, 0));
                CK(hipStreamWaitEvent(s0, j1, 0));
                CK(hipEventDestroy(j0));
                CK(hipEventDestroy(j1));
            });
        }
    // check the last copies
    unsigned char* ha = (unsigned char*)malloc(bytes);
    CK(hipMemcpy(ha, d_a, bytes, hipMemcpyDeviceToHost));
    int bad = 0;
    for (size_t i = 0; i < bytes; i++) bad |= ha[i] != 1 || ((unsigned char*)h_out)[i] != 4;
    printf("copies %s\n", bad ? "WRONG" : "ok");
    return bad;
}
