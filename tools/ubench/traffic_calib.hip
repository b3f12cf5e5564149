// traffic_calib.hip -- known-byte-count kernels for calibrating rocprofv3
// FETCH_SIZE / WRITE_SIZE on gfx950 in the RC4 kernel's own access patterns
// (MI355X_MICROARCH.md: FETCH_SIZE reads 1/2 of a wide coalesced stream; other
// widths uncalibrated).  Each kernel moves exactly BYTES bytes over a buffer
// far larger than the 256 MiB Infinity Cache.
//   calib_load_lane   : per-lane 16-B loads, lane = session (1 KiB stride)
//   calib_load_coal   : coalesced 16-B/lane loads (the guide's calibrated case)
//   calib_store_lane  : per-lane 16-B stores, lane = session
//   calib_store_quad  : quad-coalesced 16-B stores (64 B per 4 lanes)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHECK(x) do { if ((x) != hipSuccess) { printf("HIP error line %d\n", __LINE__); return 1; } } while (0)

constexpr size_t kSessions = 1u << 20;     // x 1 KiB = 1 GiB
constexpr int kBlocks = 16;                // 16 x 64 B per session

__global__ void __launch_bounds__(256) calib_load_lane(const uint4 *buf, uint32_t *sink) {
    const size_t s = (size_t)blockIdx.x * 256 + threadIdx.x;
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (int b = 0; b < kBlocks * 4; ++b) { uint4 v = buf[s * 64 + b]; acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w; }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u) sink[0] = 1;
}
__global__ void __launch_bounds__(256) calib_load_coal(const uint4 *buf, uint32_t *sink) {
    const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x, n = (size_t)gridDim.x * 256;
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (int b = 0; b < kBlocks * 4; ++b) { uint4 v = buf[b * n + t]; acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w; }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u) sink[0] = 1;
}
__global__ void __launch_bounds__(256) calib_store_lane(uint4 *buf) {
    const size_t s = (size_t)blockIdx.x * 256 + threadIdx.x;
    for (int b = 0; b < kBlocks * 4; ++b) buf[s * 64 + b] = make_uint4(b, 1, 2, 3);
}
__global__ void __launch_bounds__(256) calib_store_quad(uint4 *buf) {
    const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
    const size_t base = t & ~(size_t)63;
    const uint32_t lane = threadIdx.x & 63;
    for (int b = 0; b < kBlocks; ++b)
        for (int q = 0; q < 4; ++q) {
            const size_t sess = base + q * 16 + lane / 4;
            buf[sess * 64 + b * 4 + (lane & 3)] = make_uint4(b, q, 2, 3);
        }
}

int main() {
    uint4 *buf; uint32_t *sink;
    const size_t bytes = kSessions * 1024;
    CHECK(hipMalloc(&buf, bytes));
    CHECK(hipMalloc(&sink, 64));
    CHECK(hipMemset(buf, 1, bytes));
    const dim3 grid(kSessions / 256), blk(256);
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(calib_load_lane, grid, blk, 0, 0, buf, sink);
        hipLaunchKernelGGL(calib_load_coal, grid, blk, 0, 0, buf, sink);
        hipLaunchKernelGGL(calib_store_lane, grid, blk, 0, 0, buf);
        hipLaunchKernelGGL(calib_store_quad, grid, blk, 0, 0, buf);
    }
    CHECK(hipDeviceSynchronize());
    printf("{\"calib_bytes_per_kernel\": %zu}\n", bytes);
    return 0;
}
