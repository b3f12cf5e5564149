// ref_frame_client -- TEST INFRASTRUCTURE: a zsummerX client made of the
// REFERENCE's own frame code, whose RC4Encryption is the gfx950 mirror.
//
// oracle/Makefile (target ref-frame) compiles /root/reference/src/frame,
// src/epoll, src/timer and src/common where they lie, unchanged, with
// include/compat first on the include path, so every RC4 hook of the
// reference's TcpSession -- seeding on connect (src/frame/session.cpp:110-111),
// the recv decrypt (:313-323) and the send encrypts (:496-499, :535-538,
// :603-606) -- runs zsummerx_amd::RC4Encryption over libzrc4.so (the
// keystream reservoir, zrc4_ks_*).  This file is only the application on top:
// N connecters with SessionOptions::_rc4TcpEncryption set (config.h:196),
// each sending proto4z packets (4-byte length + 2-byte proto id + body,
// proto4z.h:704-748) and checking every echo against what it sent.
//
//   ref_frame_client --port P [--host 127.0.0.1] --key-hex K [--sessions 8]
//                    [--echoes 40] [--block 1024] [--depth 2] [--seed 1] [--seconds 60]
//
// Prints one JSON line: linked, echoes, mismatches, closed_early, bytes.
// tests/test_reference_frame.py runs it against an oracle echo server (the
// wire must be the reference's RC4) and against the engine's device hooks.
#include <zsummerX/zsummerX.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

using namespace zsummer::network;

namespace {

struct Args {
    std::string host = "127.0.0.1";
    unsigned short port = 0;
    std::string key;
    unsigned sessions = 8, echoes = 40, block = 1024, depth = 2, seed = 1, seconds = 60;
};

struct Peer {
    unsigned sent = 0, got = 0, mismatches = 0;
    bool done = false;
};

Args g_args;
std::unordered_map<SessionID, Peer> g_peers;
unsigned g_linked = 0, g_done = 0, g_closedEarly = 0;
unsigned long long g_echoes = 0, g_mismatches = 0, g_bytes = 0;

// Packet k of connecter `sid`: deterministic, `block` bytes, a proto4z frame.
std::string makePacket(SessionID sid, unsigned k)
{
    std::string p(g_args.block, '\0');
    const unsigned len = g_args.block;
    std::memcpy(&p[0], &len, 4);
    const unsigned short proto = (unsigned short)(k & 0xFFFF);
    std::memcpy(&p[4], &proto, 2);
    unsigned long long x = (g_args.seed * 0x9E3779B97F4A7C15ull) ^ ((unsigned long long)sid << 32) ^ k;
    for (unsigned i = 6; i < len; ++i) {
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        p[i] = (char)(x >> 56);
    }
    return p;
}

void sendNext(const TcpSessionPtr &s, Peer &pr)
{
    const std::string p = makePacket(s->getSessionID(), pr.sent++);
    s->send(p.data(), (unsigned)p.size());
}

void finishOne(Peer &pr)
{
    if (pr.done) return;
    pr.done = true;
    if (++g_done == g_args.sessions) SessionManager::getRef().stop();
}

bool parse(int argc, char **argv)
{
    for (int i = 1; i + 1 < argc; i += 2) {
        const std::string k = argv[i], v = argv[i + 1];
        if (k == "--host") g_args.host = v;
        else if (k == "--port") g_args.port = (unsigned short)std::atoi(v.c_str());
        else if (k == "--sessions") g_args.sessions = (unsigned)std::atoi(v.c_str());
        else if (k == "--echoes") g_args.echoes = (unsigned)std::atoi(v.c_str());
        else if (k == "--block") g_args.block = (unsigned)std::atoi(v.c_str());
        else if (k == "--depth") g_args.depth = (unsigned)std::atoi(v.c_str());
        else if (k == "--seed") g_args.seed = (unsigned)std::atoi(v.c_str());
        else if (k == "--seconds") g_args.seconds = (unsigned)std::atoi(v.c_str());
        else if (k == "--key-hex") {
            if (v.size() % 2) return false;
            g_args.key.clear();
            for (size_t j = 0; j < v.size(); j += 2) g_args.key += (char)std::strtoul(v.substr(j, 2).c_str(), nullptr, 16);
        } else {
            return false;
        }
    }
    return g_args.port && g_args.block >= 6 && g_args.block <= 20480 && g_args.depth >= 1;
}

}  // namespace

int main(int argc, char **argv)
{
    if (!parse(argc, argv)) {
        std::fprintf(stderr, "usage: ref_frame_client --port P --key-hex K [--host H] [--sessions N] [--echoes E] "
                             "[--block B<=20480] [--depth D] [--seed S] [--seconds T]\n");
        return 2;
    }
    FNLog::FastStartDefaultLogger();
    FNLog::BatchSetChannelConfig(FNLog::GetDefaultLogger(), FNLog::CHANNEL_CFG_PRIORITY, FNLog::PRIORITY_ERROR);
    SessionManager &sm = SessionManager::getRef();
    sm.start();
    for (unsigned i = 0; i < g_args.sessions; ++i) {
        const SessionID cid = sm.addConnecter(g_args.host, g_args.port);
        SessionOptions &o = sm.getConnecterOptions(cid);
        o._rc4TcpEncryption = g_args.key;          // the switch (config.h:196)
        o._reconnects = 0;
        o._onSessionLinked = [](const TcpSessionPtr &s) {
            ++g_linked;
            Peer &pr = g_peers[s->getSessionID()];
            for (unsigned d = 0; d < g_args.depth && pr.sent < g_args.echoes; ++d) sendNext(s, pr);
        };
        o._onRawPacketProc = [](const TcpSessionPtr &s, const char *begin, unsigned len) {
            Peer &pr = g_peers[s->getSessionID()];
            const std::string want = makePacket(s->getSessionID(), pr.got++);
            if (len != want.size() || std::memcmp(begin, want.data(), len) != 0) {
                ++pr.mismatches;
                ++g_mismatches;
            }
            ++g_echoes;
            g_bytes += len;
            if (pr.sent < g_args.echoes) sendNext(s, pr);
            if (pr.got == g_args.echoes) {
                finishOne(pr);
                s->close();
            }
        };
        o._onSessionClosed = [](const TcpSessionPtr &s) {
            Peer &pr = g_peers[s->getSessionID()];
            if (!pr.done) {
                ++g_closedEarly;
                finishOne(pr);
            }
        };
        if (!sm.openConnecter(cid)) {
            std::fprintf(stderr, "openConnecter failed\n");
            return 1;
        }
    }
    sm.createTimer(g_args.seconds * 1000u, [&sm]() { sm.stop(); });
    sm.run();
    std::printf("{\"linked\": %u, \"echoes\": %llu, \"mismatches\": %llu, \"closed_early\": %u, \"bytes\": %llu, "
                "\"sessions\": %u, \"expected_echoes\": %llu}\n",
                g_linked, g_echoes, g_mismatches, g_closedEarly, g_bytes, g_args.sessions,
                (unsigned long long)g_args.sessions * g_args.echoes);
    std::fflush(stdout);
    const bool ok = g_mismatches == 0 && g_closedEarly == 0 && g_echoes == (unsigned long long)g_args.sessions * g_args.echoes;
    return ok ? 0 : 1;
}
