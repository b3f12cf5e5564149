// hostmem_probe.cpp -- where does a zero-copy engine hook call spend its time?
// Times zrc4_crypt / zrc4_crypt_range on n sessions x len bytes whose payload
// sits in (a) device memory, (b) coherent pinned host memory
// (hipHostMallocDefault), (c) non-coherent pinned host memory
// (hipHostMallocNonCoherent), each through the ids path (shuffled slots) and
// the range path, averaged over R calls with HIP events; also the cost of an
// empty launch + wait.  Prints one JSON line per case.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <numeric>
#include <random>
#include <string>
#include <vector>

#include "zrc4.h"

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                                \
        }                                                                            \
    } while (0)

__global__ void empty_kernel(uint32_t *f)
{
    if (threadIdx.x == 1000) f[0] = 1;
}

__global__ void flag_kernel(uint32_t *f)
{
    if (threadIdx.x == 0) __hip_atomic_store(f, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

int main(int argc, char **argv)
{
    const uint32_t n = argc > 1 ? (uint32_t)std::stoul(argv[1]) : 2048;
    const uint32_t len = argc > 2 ? (uint32_t)std::stoul(argv[2]) : 1024;
    const int R = argc > 3 ? std::stoi(argv[3]) : 50;
    const size_t stride = 20544;                       // engine SessionBlock stride
    zrc4_ctx *ctx = nullptr;
    if (zrc4_create(&ctx, 0, n) != ZRC4_OK) return 1;
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    uint32_t *ids, *lens;
    uint64_t *offs;
    CK(hipHostMalloc((void **)&ids, n * 4, hipHostMallocDefault));
    CK(hipHostMalloc((void **)&lens, n * 4, hipHostMallocDefault));
    CK(hipHostMalloc((void **)&offs, n * 8, hipHostMallocDefault));
    std::vector<uint32_t> perm(n);
    std::iota(perm.begin(), perm.end(), 0u);
    std::shuffle(perm.begin(), perm.end(), std::mt19937(1));
    for (uint32_t i = 0; i < n; ++i) {
        lens[i] = len;
        offs[i] = (uint64_t)i * stride + 64;
    }
    const size_t bytes = (size_t)n * stride + 128;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));

    // empty round trip: a zero-entry... use a 1-entry crypt of 1 byte
    {
        uint8_t *d;
        CK(hipMalloc(&d, 64));
        uint32_t one = 1;
        uint64_t zo = 0;
        uint32_t *pid;
        CK(hipHostMalloc((void **)&pid, 4, hipHostMallocDefault));
        *pid = 0;
        uint64_t *po;
        uint32_t *pl;
        CK(hipHostMalloc((void **)&po, 8, hipHostMallocDefault));
        CK(hipHostMalloc((void **)&pl, 4, hipHostMallocDefault));
        *po = zo;
        *pl = one;
        for (int w = 0; w < 5; ++w) { zrc4_crypt(ctx, pid, d, po, pl, 1, s); zrc4_sync(ctx, s); }
        auto t0 = std::chrono::steady_clock::now();
        for (int r = 0; r < R; ++r) { zrc4_crypt(ctx, pid, d, po, pl, 1, s); zrc4_sync(ctx, s); }
        auto t1 = std::chrono::steady_clock::now();
        std::printf("{\"case\": \"1 byte, launch+sync round trip\", \"us_per_call\": %.2f}\n",
                    std::chrono::duration<double>(t1 - t0).count() * 1e6 / R);
    }

    // round-trip anatomy with an empty kernel: launch + each way of waiting
    {
        auto timeit = [&](const char *what, auto &&fn) {
            for (int w = 0; w < 5; ++w) fn();
            auto t0 = std::chrono::steady_clock::now();
            for (int r = 0; r < R; ++r) fn();
            auto t1 = std::chrono::steady_clock::now();
            std::printf("{\"case\": \"%s\", \"us_per_call\": %.2f}\n", what,
                        std::chrono::duration<double>(t1 - t0).count() * 1e6 / R);
        };
        uint32_t *hflag, *dflag;
        CK(hipHostMalloc((void **)&hflag, 4, hipHostMallocDefault));
        CK(hipMalloc((void **)&dflag, 4));
        hipEvent_t ev;
        CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        timeit("empty kernel + hipStreamSynchronize", [&]() {
            hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, dflag);
            (void)hipStreamSynchronize(s);
        });
        timeit("empty kernel + spin hipStreamQuery", [&]() {
            hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, dflag);
            while (hipStreamQuery(s) == hipErrorNotReady) {}
        });
        timeit("empty kernel + event record + hipEventSynchronize", [&]() {
            hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, dflag);
            (void)hipEventRecord(ev, s);
            (void)hipEventSynchronize(ev);
        });
        timeit("empty kernel writing a pinned flag + host spin on the flag", [&]() {
            *(volatile uint32_t *)hflag = 0;
            hipLaunchKernelGGL(flag_kernel, dim3(1), dim3(64), 0, s, hflag);
            while (*(volatile uint32_t *)hflag == 0) {}
            (void)hipStreamSynchronize(s);
        });
        timeit("empty kernel + 4-byte D2H memcpyAsync + hipStreamSynchronize", [&]() {
            hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, dflag);
            (void)hipMemcpyAsync(hflag, dflag, 4, hipMemcpyDeviceToHost, s);
            (void)hipStreamSynchronize(s);
        });
        timeit("zrc4_sync alone (nothing queued)", [&]() { (void)zrc4_sync(ctx, s); });
    }

    struct Mem { const char *name; unsigned flag; bool device; };
    const Mem mems[] = {{"device", 0, true}, {"pinned-coherent", hipHostMallocDefault, false},
                        {"pinned-noncoherent", hipHostMallocNonCoherent, false}};
    for (const Mem &m : mems) {
        uint8_t *buf = nullptr;
        if (m.device) CK(hipMalloc(&buf, bytes));
        else CK(hipHostMalloc((void **)&buf, bytes, m.flag));
        CK(hipMemset(buf, 0x5a, bytes));
        CK(hipDeviceSynchronize());
        for (int path = 0; path < 2; ++path) {
            for (uint32_t i = 0; i < n; ++i) ids[i] = path ? i : perm[i];
            auto call = [&]() {
                return path ? zrc4_crypt_range(ctx, 0, buf, offs, lens, n, s)
                            : zrc4_crypt(ctx, ids, buf, offs, lens, n, s);
            };
            for (int w = 0; w < 3; ++w) call();
            CK(hipStreamSynchronize(s));
            CK(hipEventRecord(a, s));
            for (int r = 0; r < R; ++r) call();
            CK(hipEventRecord(b, s));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            auto t0 = std::chrono::steady_clock::now();
            for (int r = 0; r < R; ++r) { call(); zrc4_sync(ctx, s); }
            auto t1 = std::chrono::steady_clock::now();
            std::printf("{\"mem\": \"%s\", \"path\": \"%s\", \"n\": %u, \"len\": %u, \"kernel_us\": %.2f, "
                        "\"call_sync_us\": %.2f, \"payload_gib_s\": %.3f}\n",
                        m.name, path ? "range" : "ids", n, len, ms * 1e3 / R,
                        std::chrono::duration<double>(t1 - t0).count() * 1e6 / R,
                        (double)n * len / (ms * 1e-3 / R) / 1073741824.0);
        }
        if (m.device) CK(hipFree(buf));
        else CK(hipHostFree(buf));
    }
    if (zrc4_sync(ctx, s) != ZRC4_OK) return 2;
    zrc4_destroy(ctx);
    return 0;
}
