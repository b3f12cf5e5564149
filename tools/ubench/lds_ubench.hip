// lds_ubench.hip -- microbenchmarks behind the RC4 kernel design (gfx950).
//
//   1. dependent-chain latency of ds_read_u8 / ds_read_b32 (one wave)
//   2. per-CU throughput (LDS cycles per wave-instruction) of the byte, dword
//      and atomic LDS ops a PRGA step could use, on the conflict-free column
//      layout of the RC4 kernel (address = row<<8 | col)
//   3. the PRGA step loop of zrc4_kernels.hpp alone (no global memory), at
//      1 wave per CU, 4 and 8 waves per CU: cycles per byte per lane
//
// Clock: s_memtime (shader clock) against s_memrealtime (100 MHz).
// Build: hipcc --offload-arch=gfx950 -O3 -o lds_ubench lds_ubench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <algorithm>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

__device__ __forceinline__ uint64_t memtime() { return __builtin_amdgcn_s_memtime(); }
__device__ __forceinline__ uint64_t realtime() { return __builtin_amdgcn_s_memrealtime(); }

__device__ __forceinline__ uint32_t col_of(uint32_t j) {
    const uint32_t w = j >> 6, l = j & 63u;
    return ((l & 31u) << 2) | (l >> 5) | ((w & 1u) << 1) | ((w >> 1) << 7);
}

// ---------------------------------------------------------------- 1. latency
template <int DWORD>
__global__ void lat_kernel(uint64_t *out, int iters) {
    __shared__ __attribute__((aligned(16))) uint8_t S[65536];
    const uint32_t col = col_of(threadIdx.x);
    for (int k = 0; k < 256; ++k) S[(k << 8) | col] = (uint8_t)((k * 73 + 11) & 255);
    __syncthreads();
    uint32_t v = 1;
    uint64_t t0 = memtime(), r0 = realtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            uint32_t a = (v << 8) | col;
            if (DWORD) asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a & ~3u));
            else asm volatile("ds_read_u8 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a));
            v &= 255u;
        }
    }
    uint64_t t1 = memtime(), r1 = realtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = r1 - r0; out[2] = v; }
}

// ------------------------------------------------------------- 2. throughput
// OP: 0 ds_read_u8, 1 ds_write_b8, 2 ds_read_b32, 3 ds_write_b32,
//     4 ds_mskor_rtn_b32, 5 ds_wrxchg_rtn_b32, 6 ds_read_u8 (random rows)
#define REP8(X) X X X X X X X X
template <int OP>
__global__ void __launch_bounds__(256) tp_kernel(uint64_t *out, int iters) {
    __shared__ __attribute__((aligned(16))) uint8_t S[65536];
    const uint32_t col = col_of(threadIdx.x);
    const uint32_t dcol = col & ~3u;
    uint32_t a0 = (((threadIdx.x * 37u) & 255u) << 8) | (OP >= 2 && OP <= 5 ? dcol : col);
    uint32_t a1 = a0 ^ 0x1100u, a2 = a0 ^ 0x2200u, a3 = a0 ^ 0x4400u;
    if (OP == 6) { a1 = a0 ^ ((threadIdx.x * 29u & 255u) << 8); a2 = a0 ^ ((threadIdx.x * 113u & 255u) << 8); a3 = a0 ^ 0x8800u; }
    uint32_t d = threadIdx.x, m = 0xFFu, r0 = 0, r1 = 0, r2 = 0, r3 = 0;
    __syncthreads();
    uint64_t t0 = memtime();
    for (int i = 0; i < iters; ++i) {
        if (OP == 0 || OP == 6)
            asm volatile(REP8("ds_read_u8 %0, %4\n\tds_read_u8 %1, %5\n\tds_read_u8 %2, %6\n\tds_read_u8 %3, %7\n\t") "s_waitcnt lgkmcnt(0)"
                         : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3) : "v"(a0), "v"(a1), "v"(a2), "v"(a3));
        if (OP == 1)
            asm volatile(REP8("ds_write_b8 %0, %4\n\tds_write_b8 %1, %4\n\tds_write_b8 %2, %4\n\tds_write_b8 %3, %4\n\t") "s_waitcnt lgkmcnt(0)"
                         :: "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(d) : "memory");
        if (OP == 2)
            asm volatile(REP8("ds_read_b32 %0, %4\n\tds_read_b32 %1, %5\n\tds_read_b32 %2, %6\n\tds_read_b32 %3, %7\n\t") "s_waitcnt lgkmcnt(0)"
                         : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3) : "v"(a0), "v"(a1), "v"(a2), "v"(a3));
        if (OP == 3)
            asm volatile(REP8("ds_write_b32 %0, %4\n\tds_write_b32 %1, %4\n\tds_write_b32 %2, %4\n\tds_write_b32 %3, %4\n\t") "s_waitcnt lgkmcnt(0)"
                         :: "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(d) : "memory");
        if (OP == 4)
            asm volatile(REP8("ds_mskor_rtn_b32 %0, %4, %8, %9\n\tds_mskor_rtn_b32 %1, %5, %8, %9\n\tds_mskor_rtn_b32 %2, %6, %8, %9\n\tds_mskor_rtn_b32 %3, %7, %8, %9\n\t") "s_waitcnt lgkmcnt(0)"
                         : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3) : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(m), "v"(d) : "memory");
        if (OP == 5)
            asm volatile(REP8("ds_wrxchg_rtn_b32 %0, %4, %8\n\tds_wrxchg_rtn_b32 %1, %5, %8\n\tds_wrxchg_rtn_b32 %2, %6, %8\n\tds_wrxchg_rtn_b32 %3, %7, %8\n\t") "s_waitcnt lgkmcnt(0)"
                         : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3) : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(d) : "memory");
    }
    uint64_t t1 = memtime();
    if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
    if (r0 + r1 + r2 + r3 == 0xdeadbeef) out[1 << 20] = 1;
}

// ----------------------------------------------------------- 3. PRGA alone
#define ZRC4_CORE(XC, XN, A, P, K)                                                               \
    "v_add_u32_sdwa %[ya], %[ya], %[" #A "] dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE "          \
    "src0_sel:BYTE_1 src1_sel:BYTE_0\n\t"                                                        \
    "ds_read_u8 %[b], %[ya]\n\t"                                                                 \
    "ds_write_b8 %[ya], %[" #A "]\n\t"                                                           \
    "v_add_u32_sdwa %[" #XN "], 1, %[" #XC "] dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE "        \
    "src0_sel:DWORD src1_sel:BYTE_1\n\t"                                                         \
    "ds_read_u8 %[" #P "], %[" #XN "]\n\t"                                                       \
    "s_waitcnt lgkmcnt(2)\n\t"                                                                   \
    "ds_write_b8 %[" #XC "], %[b]\n\t"                                                           \
    "v_add_u32_sdwa %[ta], %[" #A "], %[b] dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE "           \
    "src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"                                                        \
    "ds_read_u8 %[" #K "], %[ta]\n\t"                                                            \
    "s_waitcnt lgkmcnt(2)\n\t"
#define ZRC4_XOR(D, SEL, K)                                                                      \
    "v_xor_b32_sdwa %[" #D "], %[" #D "], %[" #K "] dst_sel:" #SEL                               \
    " dst_unused:UNUSED_PRESERVE src0_sel:" #SEL " src1_sel:BYTE_0\n\t"
#define ZE ZRC4_CORE(x0, x1, a0, a1, k0)
#define ZO ZRC4_CORE(x1, x0, a1, a0, k1)
#define ZW ZE ZRC4_XOR(d, BYTE_3, k1) ZO ZRC4_XOR(d, BYTE_0, k0) ZE ZRC4_XOR(d, BYTE_1, k1) ZO ZRC4_XOR(d, BYTE_2, k0)

__global__ void __launch_bounds__(256) prga_kernel(uint64_t *out, int iters, int active_waves) {
    __shared__ __attribute__((aligned(16))) uint8_t S[65536];
    const uint32_t col = col_of(threadIdx.x);
    for (int k = 0; k < 256; ++k) S[(k << 8) | col] = (uint8_t)((k * 73 + threadIdx.x) & 255);
    __syncthreads();
    if ((int)(threadIdx.x >> 6) >= active_waves) return;
    uint32_t ya = (7u << 8) | col, ta = col, x0 = (1u << 8) | col, x1 = col, a0 = S[x0], d = 0;
    uint32_t a1, b, k0 = 0, k1 = 0;
    uint64_t t0 = memtime(), r0 = realtime();
    for (int i = 0; i < iters; ++i) {
        asm volatile(ZW ZW ZW ZW ZW ZW ZW ZW ZW ZW ZW ZW ZW ZW ZW ZW "s_waitcnt lgkmcnt(0)\n\t"
                     : [ya] "+v"(ya), [ta] "+v"(ta), [x0] "+v"(x0), [x1] "+v"(x1), [a0] "+v"(a0),
                       [a1] "=&v"(a1), [b] "=&v"(b), [k0] "+v"(k0), [k1] "+v"(k1), [d] "+v"(d)
                     :: "memory");
    }
    uint64_t t1 = memtime(), r1 = realtime();
    if ((threadIdx.x & 63) == 0) {
        out[2 * (blockIdx.x * 4 + (threadIdx.x >> 6))] = t1 - t0;
        out[2 * (blockIdx.x * 4 + (threadIdx.x >> 6)) + 1] = r1 - r0;
    }
    if (d == 0x12345678u) out[1 << 20] = d;
}


// ------------------------------------------- 4. PRGA + payload traffic ablation
// MODE 0: per-lane session stream (lane's 64 B block at base + lane*L + blk*64,
//         L = 1 KiB: one session per lane, like crypt_kernel)
// MODE 1: coalesced (lane's 64 B at base + blk*64*256 + tid*64)
// MODE 2: loads/stores issued but no PRGA (memory path alone, per-lane pattern)
template <int MODE>
__global__ void __launch_bounds__(256) prga_mem_kernel(uint64_t *out, uint4 *buf, int nblk) {
    __shared__ __attribute__((aligned(16))) uint8_t S[65536];
    const uint32_t col = col_of(threadIdx.x);
    for (int k = 0; k < 256; ++k) S[(k << 8) | col] = (uint8_t)((k * 73 + threadIdx.x) & 255);
    __syncthreads();
    const size_t gtid = (size_t)blockIdx.x * 256 + threadIdx.x;
    uint32_t ya = (7u << 8) | col, ta = col, x0 = (1u << 8) | col, x1 = col, a0 = S[x0];
    uint32_t a1, b, k0 = 0, k1 = 0;
    uint64_t t0 = memtime();
    for (int blk = 0; blk < nblk; ++blk) {
        uint4 *p = (MODE == 1) ? buf + ((size_t)blk * gridDim.x * 256 + gtid) * 4
                               : buf + (gtid * (size_t)nblk + blk) * 4;
        uint4 v0 = p[0], v1 = p[1], v2 = p[2], v3 = p[3];
        uint32_t d[16] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w, v2.x, v2.y, v2.z, v2.w, v3.x, v3.y, v3.z, v3.w};
        if (MODE != 2) {
#define ZWD(DP, D) ZE ZRC4_XOR(DP, BYTE_3, k1) ZO ZRC4_XOR(D, BYTE_0, k0) ZE ZRC4_XOR(D, BYTE_1, k1) ZO ZRC4_XOR(D, BYTE_2, k0)
            asm volatile(ZWD(d15, d0) ZWD(d0, d1) ZWD(d1, d2) ZWD(d2, d3) ZWD(d3, d4) ZWD(d4, d5) ZWD(d5, d6) ZWD(d6, d7)
                         ZWD(d7, d8) ZWD(d8, d9) ZWD(d9, d10) ZWD(d10, d11) ZWD(d11, d12) ZWD(d12, d13) ZWD(d13, d14) ZWD(d14, d15)
                         "s_waitcnt lgkmcnt(0)\n\t"
                         : [ya] "+v"(ya), [ta] "+v"(ta), [x0] "+v"(x0), [x1] "+v"(x1), [a0] "+v"(a0),
                           [a1] "=&v"(a1), [b] "=&v"(b), [k0] "+v"(k0), [k1] "+v"(k1),
                           [d0] "+v"(d[0]), [d1] "+v"(d[1]), [d2] "+v"(d[2]), [d3] "+v"(d[3]),
                           [d4] "+v"(d[4]), [d5] "+v"(d[5]), [d6] "+v"(d[6]), [d7] "+v"(d[7]),
                           [d8] "+v"(d[8]), [d9] "+v"(d[9]), [d10] "+v"(d[10]), [d11] "+v"(d[11]),
                           [d12] "+v"(d[12]), [d13] "+v"(d[13]), [d14] "+v"(d[14]), [d15] "+v"(d[15])
                         :: "memory");
        } else {
#pragma unroll
            for (int q = 0; q < 16; ++q) d[q] ^= 0x5au;
        }
        p[0] = make_uint4(d[0], d[1], d[2], d[3]); p[1] = make_uint4(d[4], d[5], d[6], d[7]);
        p[2] = make_uint4(d[8], d[9], d[10], d[11]); p[3] = make_uint4(d[12], d[13], d[14], d[15]);
    }
    uint64_t t1 = memtime();
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}


// ---------------------------------------- 5. payload access-pattern ablation
// Memory path alone (xor 0x5a), one block of prefetch, 8 waves/CU, 4 rounds.
//  PAT 0: lane = session, session stride STRIDE, lane reads its own 64 B
//  PAT 1: quad-coalesced: lanes 4g..4g+3 read 64 contiguous B of ONE session
//         (4 instructions cover sessions 4g..4g+3)
//  PAT 2: fully coalesced (consecutive lanes, consecutive 16 B)
template <int PAT>
__global__ void __launch_bounds__(256) mem_kernel(uint64_t *out, uint8_t *buf, int nblk, int stride) {
    const size_t gtid = (size_t)blockIdx.x * 256 + threadIdx.x;
    const size_t nthreads = (size_t)gridDim.x * 256;
    auto addr = [&](int blk, int q) -> uint4 * {
        if (PAT == 0) return (uint4 *)(buf + gtid * stride + blk * 64 + q * 16);
        if (PAT == 1) {  // instruction q serves session (gtid & ~3) + q; lane c = gtid&3 reads chunk c
            const size_t sess = (gtid & ~(size_t)3) + q;
            return (uint4 *)(buf + sess * stride + blk * 64 + (gtid & 3) * 16);
        }
        return (uint4 *)(buf + ((size_t)blk * nthreads * 4 + q * nthreads + gtid) * 16);
    };
    uint64_t t0 = memtime();
    uint4 c[4], n[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) c[q] = *addr(0, q);
    for (int blk = 0; blk < nblk; ++blk) {
        const int nb = blk + 1 < nblk ? blk + 1 : blk;
#pragma unroll
        for (int q = 0; q < 4; ++q) n[q] = *addr(nb, q);
#pragma unroll
        for (int q = 0; q < 4; ++q) { c[q].x ^= 0x5a; c[q].y ^= 0x5a; c[q].z ^= 0x5a; c[q].w ^= 0x5a; *addr(blk, q) = c[q]; }
#pragma unroll
        for (int q = 0; q < 4; ++q) c[q] = n[q];
    }
    uint64_t t1 = memtime();
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}


// ------------------------------- 6. load-only / store-only / DMA addressing cost
// 8 waves/CU, each lane streams 16 B accesses; session stride 1 KiB.
//  K 0: scattered dwordx4 loads (lane = session)      K 1: scattered dwordx4 stores
//  K 2: quad-coalesced dwordx4 loads                  K 3: quad-coalesced dwordx4 stores
//  K 4: quad-coalesced global_load_lds_dwordx4 (LDS-DMA, 4 KiB staging per wave)
template <int K>
__global__ void __launch_bounds__(256) addr_kernel(uint64_t *out, uint8_t *buf, int nblk) {
    __shared__ __attribute__((aligned(16))) uint8_t stage[16384];
    const size_t gtid = (size_t)blockIdx.x * 256 + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (int blk = 0; blk < nblk; ++blk) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            uint8_t *p;
            if (K == 0 || K == 1) p = buf + gtid * 1024 + blk * 64 + q * 16;
            else p = buf + ((gtid & ~(size_t)63) + q * 16 + lane / 4) * 1024 + blk * 64 + (lane & 3) * 16;
            if (K == 0 || K == 2) { uint4 v = *(uint4 *)p; acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w; }
            if (K == 1 || K == 3) *(uint4 *)p = make_uint4(blk, q, lane, 7);
            if (K == 5) {   // oct-coalesced: 8 lanes write 128 contiguous B of one session (2 blocks)
                uint8_t *po = buf + ((gtid & ~(size_t)63) + q * 8 + lane / 8 + (blk & 1) * 32) * 1024 + (blk >> 1) * 128 + (lane & 7) * 16;
                *(uint4 *)po = make_uint4(blk, q, lane, 7);
            }
            if (K == 6) {   // full-line per lane pair... 16 lanes x 64 B: 1 KiB contiguous (one session per instruction)
                uint8_t *pf = buf + ((gtid & ~(size_t)63) + q * 16 + (blk % 16)) * 1024 + lane * 16;
                *(uint4 *)pf = make_uint4(blk, q, lane, 7);
            }
            if (K == 4) __builtin_amdgcn_global_load_lds((const void *)p, (void *)(stage + wave * 4096 + q * 1024), 16, 0, 0);
        }
        if (K == 4 && (blk & 7) == 7) { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); acc.x ^= stage[threadIdx.x * 16]; }
    }
    if (acc.x == 0x12345 && acc.y == 7) out[1 << 20] = acc.z;
}

static double median(std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; }

int main() {
    uint64_t *d_out;
    CHECK(hipMalloc(&d_out, (8 << 20) + 64));
    std::vector<uint64_t> h(8192 * 2);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
    int ncu = 0; CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    printf("{\"cus\": %d,\n", ncu);

    // 1. latency
    for (int dw = 0; dw < 2; ++dw) {
        const int iters = 4096;
        if (dw) hipLaunchKernelGGL(lat_kernel<1>, dim3(1), dim3(64), 0, 0, d_out, iters);
        else hipLaunchKernelGGL(lat_kernel<0>, dim3(1), dim3(64), 0, 0, d_out, iters);
        CHECK(hipDeviceSynchronize());
        CHECK(hipMemcpy(h.data(), d_out, 24, hipMemcpyDeviceToHost));
        double cyc = (double)h[0] / (iters * 16.0);
        double ghz = (double)h[0] / ((double)h[1] * 10.0);
        printf(" \"latency_%s_cycles\": %.1f, \"latency_clock_ghz_%s\": %.3f,\n", dw ? "ds_read_b32" : "ds_read_u8", cyc,
               dw ? "b32" : "u8", ghz);
    }

    // 2. throughput: 2 WGs/CU of 256 threads (8 waves/CU), and 4 waves/CU
    const char *names[] = {"ds_read_u8", "ds_write_b8", "ds_read_b32", "ds_write_b32",
                           "ds_mskor_rtn_b32", "ds_wrxchg_rtn_b32", "ds_read_u8_rand"};
    for (int wgs = 1; wgs <= 2; ++wgs) {
        for (int op = 0; op < 7; ++op) {
            const int iters = 2000, blocks = ncu * wgs;
            auto launch = [&]() {
                switch (op) {
                case 0: hipLaunchKernelGGL(tp_kernel<0>, dim3(blocks), dim3(256), 0, 0, d_out, iters); break;
                case 1: hipLaunchKernelGGL(tp_kernel<1>, dim3(blocks), dim3(256), 0, 0, d_out, iters); break;
                case 2: hipLaunchKernelGGL(tp_kernel<2>, dim3(blocks), dim3(256), 0, 0, d_out, iters); break;
                case 3: hipLaunchKernelGGL(tp_kernel<3>, dim3(blocks), dim3(256), 0, 0, d_out, iters); break;
                case 4: hipLaunchKernelGGL(tp_kernel<4>, dim3(blocks), dim3(256), 0, 0, d_out, iters); break;
                case 5: hipLaunchKernelGGL(tp_kernel<5>, dim3(blocks), dim3(256), 0, 0, d_out, iters); break;
                case 6: hipLaunchKernelGGL(tp_kernel<6>, dim3(blocks), dim3(256), 0, 0, d_out, iters); break;
                }
            };
            launch();
            CHECK(hipDeviceSynchronize());
            CHECK(hipEventRecord(e0));
            launch();
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
            CHECK(hipMemcpy(h.data(), d_out, blocks * 8, hipMemcpyDeviceToHost));
            std::vector<double> cyc; for (int b = 0; b < blocks; ++b) cyc.push_back((double)h[b]);
            // LDS cycles per wave-instruction on one CU: per-CU instr = wgs*4 waves * iters*32
            double instr_per_cu = wgs * 4.0 * iters * 32.0;
            printf(" \"tp_%s_%dwaves\": {\"cycles_per_wave_instr\": %.2f, \"ms\": %.3f},\n", names[op], wgs * 4,
                   median(cyc) / instr_per_cu, ms);
        }
    }

    // 3. PRGA loop alone
    struct Cfg { int blocks_per_cu; int waves; const char *name; };
    Cfg cfgs[] = {{0, 1, "1wave_total"}, {1, 1, "1wave_per_cu"}, {1, 4, "4waves_per_cu"}, {2, 4, "8waves_per_cu"}};
    for (auto &c : cfgs) {
        const int iters = 64;  // x 64 bytes
        const int blocks = c.blocks_per_cu ? ncu * c.blocks_per_cu : 1;
        hipLaunchKernelGGL(prga_kernel, dim3(blocks), dim3(256), 0, 0, d_out, iters, c.waves);
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(prga_kernel, dim3(blocks), dim3(256), 0, 0, d_out, iters, c.waves);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
        CHECK(hipMemcpy(h.data(), d_out, blocks * 4 * 16, hipMemcpyDeviceToHost));
        std::vector<double> cyc, ghz;
        for (int b = 0; b < blocks; ++b)
            for (int w = 0; w < c.waves; ++w) {
                cyc.push_back((double)h[2 * (b * 4 + w)] / (iters * 64.0));
                ghz.push_back((double)h[2 * (b * 4 + w)] / ((double)h[2 * (b * 4 + w) + 1] * 10.0));
            }
        double bytes = (double)blocks * c.waves * 64 * iters * 64;
        printf(" \"prga_%s\": {\"cycles_per_byte\": %.1f, \"clock_ghz\": %.3f, \"ms\": %.4f, \"GBps\": %.1f},\n", c.name,
               median(cyc), median(ghz), ms, bytes / (ms * 1e-3) / 1e9);
    }

    // 4. PRGA + payload traffic (8 waves/CU, L = 1 KiB per lane, 4 rounds of the grid)
    {
        const int nblk = 16, blocks = ncu * 2 * 4;   // 2 WG/CU resident, 4 rounds
        uint4 *buf; CHECK(hipMalloc(&buf, (size_t)blocks * 256 * nblk * 64));
        CHECK(hipMemset(buf, 1, (size_t)blocks * 256 * nblk * 64));
        const char *mn[] = {"per_lane_session", "coalesced", "memory_only"};
        for (int mode = 0; mode < 3; ++mode) {
            auto launch = [&]() {
                if (mode == 0) hipLaunchKernelGGL(prga_mem_kernel<0>, dim3(blocks), dim3(256), 0, 0, d_out, buf, nblk);
                if (mode == 1) hipLaunchKernelGGL(prga_mem_kernel<1>, dim3(blocks), dim3(256), 0, 0, d_out, buf, nblk);
                if (mode == 2) hipLaunchKernelGGL(prga_mem_kernel<2>, dim3(blocks), dim3(256), 0, 0, d_out, buf, nblk);
            };
            launch(); CHECK(hipDeviceSynchronize());
            CHECK(hipEventRecord(e0)); launch(); CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
            float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
            CHECK(hipMemcpy(h.data(), d_out, blocks * 4 * 8, hipMemcpyDeviceToHost));
            std::vector<double> cyc; for (int b = 0; b < blocks * 4; ++b) cyc.push_back((double)h[b] / (nblk * 64.0));
            double bytes = (double)blocks * 256 * nblk * 64;
            printf(" \"prga_mem_%s\": {\"cycles_per_byte_per_wave\": %.1f, \"ms\": %.4f, \"payload_GBps\": %.1f},\n", mn[mode],
                   median(cyc), ms, bytes / (ms * 1e-3) / 1e9);
        }
        CHECK(hipFree(buf));
    }

    // 5. access-pattern ablation
    {
        const int nblk = 16, blocks = ncu * 2 * 4;
        const size_t sessions = (size_t)blocks * 256;
        uint8_t *buf; CHECK(hipMalloc(&buf, sessions * 1536 + 4096));
        CHECK(hipMemset(buf, 1, sessions * 1536 + 4096));
        struct P { int pat, stride; const char *name; };
        P ps[] = {{0, 1024, "lane_session_s1024"}, {0, 1088, "lane_session_s1088"}, {0, 1152, "lane_session_s1152"},
                  {0, 1280, "lane_session_s1280"}, {0, 1040, "lane_session_s1040"},
                  {1, 1024, "quad_coalesced_s1024"}, {1, 1088, "quad_coalesced_s1088"}, {2, 1024, "coalesced"}};
        for (auto &p : ps) {
            auto launch = [&]() {
                if (p.pat == 0) hipLaunchKernelGGL(mem_kernel<0>, dim3(blocks), dim3(256), 0, 0, d_out, buf, nblk, p.stride);
                if (p.pat == 1) hipLaunchKernelGGL(mem_kernel<1>, dim3(blocks), dim3(256), 0, 0, d_out, buf, nblk, p.stride);
                if (p.pat == 2) hipLaunchKernelGGL(mem_kernel<2>, dim3(blocks), dim3(256), 0, 0, d_out, buf, nblk, p.stride);
            };
            launch(); CHECK(hipDeviceSynchronize());
            CHECK(hipEventRecord(e0)); launch(); CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
            float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
            double bytes = (double)sessions * nblk * 64;
            printf(" \"mem_%s\": {\"ms\": %.4f, \"payload_GBps\": %.1f, \"rw_GBps\": %.1f},\n", p.name, ms,
                   bytes / (ms * 1e-3) / 1e9, 2 * bytes / (ms * 1e-3) / 1e9);
        }
        CHECK(hipFree(buf));
    }

    // 6. addressing cost of scattered vs quad-coalesced loads/stores and LDS-DMA
    {
        const int nblk = 16, blocks = ncu * 2 * 4;
        const size_t sessions = (size_t)blocks * 256;
        uint8_t *buf; CHECK(hipMalloc(&buf, sessions * 1024 + 4096));
        CHECK(hipMemset(buf, 1, sessions * 1024 + 4096));
        const char *kn[] = {"scatter_load", "scatter_store", "quad_load", "quad_store", "quad_lds_dma_load", "oct_store", "kib_store"};
        for (int kk = 0; kk < 7; ++kk) {
            auto launch = [&]() {
                switch (kk) {
                case 0: hipLaunchKernelGGL(addr_kernel<0>, dim3(blocks), dim3(256), 0, 0, d_out, buf, nblk); break;
                case 1: hipLaunchKernelGGL(addr_kernel<1>, dim3(blocks), dim3(256), 0, 0, d_out, buf, nblk); break;
                case 2: hipLaunchKernelGGL(addr_kernel<2>, dim3(blocks), dim3(256), 0, 0, d_out, buf, nblk); break;
                case 3: hipLaunchKernelGGL(addr_kernel<3>, dim3(blocks), dim3(256), 0, 0, d_out, buf, nblk); break;
                case 4: hipLaunchKernelGGL(addr_kernel<4>, dim3(blocks), dim3(256), 0, 0, d_out, buf, nblk); break;
                case 5: hipLaunchKernelGGL(addr_kernel<5>, dim3(blocks), dim3(256), 0, 0, d_out, buf, nblk); break;
                case 6: hipLaunchKernelGGL(addr_kernel<6>, dim3(blocks), dim3(256), 0, 0, d_out, buf, nblk); break;
                }
            };
            launch(); CHECK(hipDeviceSynchronize());
            CHECK(hipEventRecord(e0)); launch(); CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
            float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
            double bytes = (double)sessions * nblk * 64;
            double instr_per_cu = (double)blocks * 4 * nblk * 4 / ncu;   // wave-instructions per CU
            printf(" \"addr_%s\": {\"ms\": %.4f, \"GBps\": %.1f, \"ns_per_wave_instr_per_cu\": %.2f},\n", kn[kk], ms,
                   bytes / (ms * 1e-3) / 1e9, ms * 1e6 / instr_per_cu);
        }
        CHECK(hipFree(buf));
    }
    printf(" \"done\": 1}\n");
    return 0;
}
