// mirror_bench.cpp -- per-call cost of the drop-in RC4Encryption mirror
// (include/zsummerx_amd/rc4_encryption.h) under the reference's call pattern:
// TcpSession::onRecv / send call encryption() once per block
// (src/frame/session.cpp:323, :498, :537, :605).  `sessions` pairs of streams
// (client write -> server read, same key) exchange `bytes`-byte blocks for
// `seconds`; every block is checked after the round trip.  Prints one JSON
// line.  $ZSX_RC4_RING picks the keystream reservoir's ring (0 = every call
// crypts on the device).
//
//   g++ -O2 -std=c++17 -Iinclude tools/mirror_bench.cpp -Lzsummerx_amd -lzrc4 \
//       -Wl,-rpath,$PWD/zsummerx_amd -o tools/bin/mirror_bench
//   tools/bin/mirror_bench [sessions=2] [bytes=1024] [seconds=2]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "zsummerx_amd/rc4_encryption.h"

using zsummerx_amd::RC4Encryption;

int main(int argc, char **argv)
{
    const int sessions = argc > 1 ? std::atoi(argv[1]) : 2;
    const int bytes = argc > 2 ? std::atoi(argv[2]) : 1024;
    const double seconds = argc > 3 ? std::atof(argv[3]) : 2.0;
    std::vector<RC4Encryption> cw(sessions), sr(sessions);
    for (int i = 0; i < sessions; ++i) {
        const std::string key = "bench-key-" + std::to_string(i);
        cw[i].makeSBox(key);
        sr[i].makeSBox(key);
    }
    std::vector<unsigned char> plain(bytes), wire(bytes);
    for (int j = 0; j < bytes; ++j) plain[j] = (unsigned char)(j * 31 + 7);
    long calls = 0, bad = 0;
    auto run = [&](double secs) {
        const auto t0 = std::chrono::steady_clock::now();
        long n = 0;
        for (;;) {
            for (int i = 0; i < sessions; ++i) {
                std::memcpy(wire.data(), plain.data(), bytes);
                cw[i].encryption(wire.data(), bytes);       // send side
                sr[i].encryption(wire.data(), bytes);       // receive side
                bad += std::memcmp(wire.data(), plain.data(), bytes) != 0;
                n += 2;
            }
            const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            if (el >= secs) return std::make_pair(n, el);
        }
    };
    run(0.3);                                               // warm: first calls crypt on the device
    bad = 0;
    const auto r = run(seconds);
    calls = r.first;
    const char *ring = std::getenv("ZSX_RC4_RING");
    std::printf("{\"bench\": \"mirror_per_call\", \"sessions\": %d, \"bytes\": %d, \"ring\": %s, \"calls_per_s\": %.0f, "
                "\"us_per_call\": %.3f, \"mb_per_s\": %.1f, \"mismatches\": %ld}\n",
                sessions, bytes, ring ? ring : "8192", calls / r.second, 1e6 * r.second / calls,
                calls * (double)bytes / r.second / 1e6, bad);
    return bad ? 1 : 0;
}
