// wide_ubench.hip -- PRGA with 4-byte S-box entries (one wave per 64 KiB LDS
// region, entry k of lane l at (k << 8) | (l << 2)) where b = S[y]; S[y] = a
// is ONE ds_wrxchg_rtn_b32, against the shipped byte-entry step (zrc4_kernels.hpp
// xor64_asm).  Per byte: wide = 4 LDS ops + 4 VALU + 2 waits, byte = 5 LDS ops.
// Correctness: every checked lane's keystream against a host RC4.
//   build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I. tools/ubench/wide_ubench.hip -o tools/ubench/wide_ubench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "zsummerx_amd/csrc/zrc4_kernels.hpp"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)
using namespace zrc4;

__device__ __forceinline__ uint64_t memtime() { return __builtin_amdgcn_s_memtime(); }

__host__ __device__ inline void key_of(uint32_t lane, uint8_t (&k)[8])
{
    uint32_t h = lane * 2654435761u + 12345u;
    for (int i = 0; i < 8; ++i) { h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15; k[i] = (uint8_t)h; }
}

// wide step: XC/XN = addresses of S[x] / S[x+1] (ping-pong), A = a, P <- next a, K <- keystream
#define ZW_CORE(XC, XN, A, P, K)                                                                 \
    "v_add_u32_sdwa %[ya], %[ya], %[" #A "] dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE "          \
    "src0_sel:BYTE_1 src1_sel:BYTE_0\n\t"                                                        \
    "ds_wrxchg_rtn_b32 %[b], %[ya], %[" #A "]\n\t"                                               \
    "v_add_u32_sdwa %[" #XN "], 1, %[" #XC "] dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE "        \
    "src0_sel:DWORD src1_sel:BYTE_1\n\t"                                                         \
    "ds_read_b32 %[" #P "], %[" #XN "]\n\t"                                                      \
    "s_waitcnt lgkmcnt(1)\n\t"                                                                   \
    "ds_write_b32 %[" #XC "], %[b]\n\t"                                                          \
    "v_add_u32_sdwa %[ta], %[" #A "], %[b] dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE "           \
    "src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"                                                        \
    "ds_read_b32 %[" #K "], %[ta]\n\t"                                                           \
    "s_waitcnt lgkmcnt(2)\n\t"
#define ZW_E ZW_CORE(x0, x1, a0, a1, k0)
#define ZW_O ZW_CORE(x1, x0, a1, a0, k1)
#define ZW_W0(D) ZW_E ZW_O ZRC4_XOR(D, BYTE_0, k0) ZW_E ZRC4_XOR(D, BYTE_1, k1) ZW_O ZRC4_XOR(D, BYTE_2, k0)
#define ZW_W(DP, D) ZW_E ZRC4_XOR(DP, BYTE_3, k1) ZW_O ZRC4_XOR(D, BYTE_0, k0)                    \
    ZW_E ZRC4_XOR(D, BYTE_1, k1) ZW_O ZRC4_XOR(D, BYTE_2, k0)

__device__ __forceinline__ void xor64_wide(Rc4Lane &st, uint4 (&q)[4])
{
    uint32_t b, k0, k1, a1;
    asm volatile(
        ZW_W0(d0) ZW_W(d0, d1) ZW_W(d1, d2) ZW_W(d2, d3)
        ZW_W(d3, d4) ZW_W(d4, d5) ZW_W(d5, d6) ZW_W(d6, d7)
        ZW_W(d7, d8) ZW_W(d8, d9) ZW_W(d9, d10) ZW_W(d10, d11)
        ZW_W(d11, d12) ZW_W(d12, d13) ZW_W(d13, d14) ZW_W(d14, d15)
        "s_waitcnt lgkmcnt(0)\n\t"
        ZRC4_XOR(d15, BYTE_3, k1)
        : [ya] "+v"(st.ya), [ta] "+v"(st.ta), [x0] "+v"(st.x0), [x1] "+v"(st.x1),
          [a0] "+v"(st.a0), [a1] "=&v"(a1), [b] "=&v"(b), [k0] "=&v"(k0), [k1] "=&v"(k1),
          [d0] "+v"(q[0].x), [d1] "+v"(q[0].y), [d2] "+v"(q[0].z), [d3] "+v"(q[0].w),
          [d4] "+v"(q[1].x), [d5] "+v"(q[1].y), [d6] "+v"(q[1].z), [d7] "+v"(q[1].w),
          [d8] "+v"(q[2].x), [d9] "+v"(q[2].y), [d10] "+v"(q[2].z), [d11] "+v"(q[2].w),
          [d12] "+v"(q[3].x), [d13] "+v"(q[3].y), [d14] "+v"(q[3].z), [d15] "+v"(q[3].w)
        :
        : "memory");
}

// MODE 0: byte entries, 256-thread block (4 waves share a 64 KiB image)
// MODE 1: wide entries, 64-thread block (one wave, 64 KiB) -- 1 or 2 blocks per CU
template <int MODE>
__global__ void __launch_bounds__(MODE ? 64 : 256) prga_kernel(uint4 *out, uint64_t *cyc, int nblk, int active_waves)
{
    __shared__ __attribute__((aligned(16))) uint32_t S32[16384];
    uint8_t *S8 = reinterpret_cast<uint8_t *>(S32);
    const uint32_t t = threadIdx.x;
    const uint32_t lane = blockIdx.x * blockDim.x + t;
    const uint32_t col = MODE ? (t << 2) : col_of(t);
    uint8_t key[8];
    key_of(lane, key);
    auto at = [&](uint32_t k) -> uint32_t { return (k << 8) | col; };
    for (int k = 0; k < 256; ++k) { if (MODE) S32[at(k) >> 2] = k; else S8[at(k)] = (uint8_t)k; }
    uint32_t j = 0;
    for (int i = 0; i < 256; ++i) {
        const uint32_t si = MODE ? S32[at(i) >> 2] : S8[at(i)];
        j = (j + si + key[i & 7]) & 255u;
        const uint32_t sj = MODE ? S32[at(j) >> 2] : S8[at(j)];
        if (MODE) { S32[at(i) >> 2] = sj; S32[at(j) >> 2] = si; } else { S8[at(i)] = (uint8_t)sj; S8[at(j)] = (uint8_t)si; }
    }
    __syncthreads();
    if ((int)(t >> 6) >= active_waves) return;
    Rc4Lane st;
    st.col = col;
    st.x0 = (1u << 8) | col;
    st.a0 = MODE ? S32[st.x0 >> 2] : S8[st.x0];
    st.ya = col;
    st.ta = col;
    st.x1 = col;
    uint4 *o = out + (size_t)lane * nblk * 4;
    const uint64_t t0 = memtime();
    for (int b = 0; b < nblk; ++b) {
        uint4 q[4] = {};
        if (MODE) xor64_wide(st, q); else xor64_asm(st, q);
        store64(o + b * 4, q);
    }
    const uint64_t t1 = memtime();
    if ((t & 63) == 0) cyc[blockIdx.x * 4 + (t >> 6)] = t1 - t0;
}

static void host_keystream(uint32_t lane, uint8_t *ks, int n)
{
    uint8_t key[8];
    key_of(lane, key);
    uint8_t S[256];
    for (int i = 0; i < 256; ++i) S[i] = (uint8_t)i;
    uint32_t j = 0;
    for (int i = 0; i < 256; ++i) { j = (j + S[i] + key[i & 7]) & 255u; uint8_t t = S[i]; S[i] = S[j]; S[j] = t; }
    uint32_t x = 0, y = 0;
    for (int i = 0; i < n; ++i) {
        x = (x + 1) & 255u; uint8_t a = S[x]; y = (y + a) & 255u; uint8_t b = S[y];
        S[x] = b; S[y] = a; ks[i] = S[(a + b) & 255u];
    }
}

int main(int argc, char **argv)
{
    const int nblk = argc > 1 ? atoi(argv[1]) : 64;
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const size_t lanes_max = (size_t)2 * cus * 256, bytes = (size_t)nblk * 64;
    uint4 *d_out; uint64_t *d_cyc;
    CHECK(hipMalloc(&d_out, lanes_max * bytes));
    CHECK(hipMalloc(&d_cyc, 2 * cus * 4 * sizeof(uint64_t)));
    std::vector<uint8_t> h(lanes_max * bytes), ref(bytes);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
    // name, mode, blocks, threads, waves per block
    struct Cfg { const char *name; int mode, blocks, threads, waves; } cfgs[] = {
        {"byte_1wave_per_cu", 0, cus, 256, 1}, {"byte_4waves_per_cu", 0, cus, 256, 4},
        {"byte_8waves_per_cu", 0, 2 * cus, 256, 4},
        {"wide_1wave_per_cu", 1, cus, 64, 1}, {"wide_2waves_per_cu", 1, 2 * cus, 64, 1}};
    printf("{\n");
    int bad_total = 0;
    for (const Cfg &c : cfgs) {
        float best = 1e30f;
        std::vector<uint64_t> cy((size_t)c.blocks * 4);
        for (int rep = 0; rep < 4; ++rep) {
            CHECK(hipMemset(d_out, 0, lanes_max * bytes));
            CHECK(hipEventRecord(e0));
            if (c.mode == 0) hipLaunchKernelGGL(prga_kernel<0>, dim3(c.blocks), dim3(c.threads), 0, 0, d_out, d_cyc, nblk, c.waves);
            else hipLaunchKernelGGL(prga_kernel<1>, dim3(c.blocks), dim3(c.threads), 0, 0, d_out, d_cyc, nblk, c.waves);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best) best = ms;
        }
        CHECK(hipMemcpy(cy.data(), d_cyc, cy.size() * 8, hipMemcpyDeviceToHost));
        double mean = 0; int nw = 0;
        for (int b = 0; b < c.blocks; ++b) for (int w = 0; w < c.waves; ++w) { mean += cy[(size_t)b * 4 + w]; ++nw; }
        mean /= nw;
        CHECK(hipMemcpy(h.data(), d_out, (size_t)c.blocks * c.threads * bytes, hipMemcpyDeviceToHost));
        int bad = 0, checked = 0;
        for (int b = 0; b < c.blocks; ++b) {
            if (b >= 8 && (b % 37) != 0) continue;
            for (int t = 0; t < c.waves * 64; ++t) {
                const uint32_t lane = b * c.threads + t;
                host_keystream(lane, ref.data(), (int)bytes);
                if (memcmp(ref.data(), h.data() + (size_t)lane * bytes, bytes) != 0) ++bad;
                ++checked;
            }
        }
        bad_total += bad;
        printf(" \"%s\": {\"cycles_per_byte\": %.2f, \"ms\": %.4f, \"checked_lanes\": %d, \"bad_lanes\": %d},\n",
               c.name, mean / bytes, best, checked, bad);
    }
    printf(" \"bad_total\": %d\n}\n", bad_total);
    return bad_total ? 2 : 0;
}
