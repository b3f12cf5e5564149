// emu_declared_check.cpp -- TEST INFRASTRUCTURE ONLY (tests/test_hooks.py).
// The CPU emulation of zrc4_crypt_grouped_declared (emu_zrc4_hip.cpp) must
// refuse what the GPU refuses (include/zrc4.h): a bucket whose
// ids leave its declared group is refused at any size; above 256 buckets
// (the GPU's declared-check kernel) its ids also block the groups they name,
// so the bucket that legitimately declares such a group is refused too.
// Prints one line per case and exits non-zero on any mismatch.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "zrc4.h"

static bool ran(const std::vector<uint8_t> &pay, uint32_t e)
{
    for (int k = 0; k < 8; ++k)
        if (pay[(size_t)e * 8 + k]) return true;
    return false;
}

static int one_case(uint32_t nb)
{
    const uint32_t groups = nb + 8, n = nb * 256;
    zrc4_ctx *c = nullptr;
    if (zrc4_create(&c, 0, groups * 256) != ZRC4_OK) return 1;
    std::vector<uint32_t> ids(n, ZRC4_IDLE_SLOT), bg(nb);
    std::vector<uint64_t> off(n);
    std::vector<uint32_t> len(n, 8);
    for (uint32_t b = 0; b < nb; ++b) {
        bg[b] = b;                                          // bucket b declares group b
        for (uint32_t k = 0; k < 4; ++k) ids[b * 256 + k] = b * 256 + k;
    }
    // bucket 3 declares group 3 but its ids lie in group 7 (slots bucket 7 does not use)
    for (uint32_t k = 0; k < 4; ++k) ids[3 * 256 + k] = 7 * 256 + 100 + k;
    for (uint32_t e = 0; e < n; ++e) off[e] = (uint64_t)e * 8;
    std::vector<uint8_t> pay((size_t)n * 8, 0);
    const int rc = zrc4_crypt_grouped_declared(c, ids.data(), bg.data(), pay.data(), off.data(), len.data(), n,
                                               nullptr, nullptr);
    const bool r3 = ran(pay, 3 * 256), r7 = ran(pay, 7 * 256), r9 = ran(pay, 9 * 256);
    const bool want7 = nb <= 256;
    const bool ok = rc == ZRC4_ERR_GROUP && !r3 && r7 == want7 && r9;
    printf("buckets %u: rc %d, bucket 3 %s, bucket 7 %s (want %s), bucket 9 %s -> %s\n", nb, rc, r3 ? "ran" : "refused",
           r7 ? "ran" : "refused", want7 ? "ran" : "refused", r9 ? "ran" : "refused", ok ? "ok" : "MISMATCH");
    zrc4_destroy(c);
    return ok ? 0 : 1;
}

int main()
{
    int bad = 0;
    for (uint32_t nb : {20u, 200u, 256u, 257u, 700u}) bad += one_case(nb);
    return bad ? 1 : 0;
}
