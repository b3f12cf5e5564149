// frame_stress.cpp -- BASELINE config 1 driver: the reference's
// example/frameStressTest (FrameStressMain.cpp) ping-pong echo over the
// batched session engine (include/zsummerx_amd/frame.h), RC4 on.
//
//   client: on link, send one proto4z packet (8-byte header + body,
//           FrameStressMain.cpp:114-122); on every echo, check it and send
//           the next (:124-170, "ping-pong" mode, --depth packets in flight
//           like g_concExtraSend);
//   server: echo every packet back (CStressServerHandler::onMessage, :263-276).
//
// Modes: loopback (server + clients in ONE engine / event loop, the default),
// server (prints "PORT <n>", serves until --seconds or --exit-after closes),
// client (--port P).  RC4 hooks: --rc4 device (the gfx950 product path,
// keystream reservoirs of --ring bytes per stream) | device-direct (one crypt
// launch over the spans per iteration) |
// host:<lib> (a CPU RC4Encryption loaded from <lib> -- oracle/liboracle.so or
// oracle/_ref/libzrc4_ref.so; tests and the CPU baseline only) | off.
// Prints one JSON line of counters.
#include <dlfcn.h>
#include <signal.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "zrc4.h"
#include "zsummerx_amd/frame.h"

using namespace zsummerx_amd;
using namespace zsummerx_amd::frame;

namespace {

// CPU RC4Encryption behind the Rc4Hooks interface, one reference-layout
// state (int x, y, box[256]; rc4_encryption.h:96-98) per slot, called once per
// span exactly as the reference hooks call it.  Test / baseline use only.
class HostLibHooks final : public Rc4Hooks {
public:
    HostLibHooks(const std::string &lib, uint32_t capacity) : states_((size_t)capacity * 258)
    {
        h_ = dlopen(lib.c_str(), RTLD_NOW | RTLD_LOCAL);
        if (!h_) throw std::runtime_error("dlopen " + lib + ": " + dlerror());
        if (void *f = dlsym(h_, "zrc4_ref_make_sbox")) {       // the real header (oracle/_ref)
            mk_ = reinterpret_cast<MakeFn>(f);
            encI_ = reinterpret_cast<EncIntFn>(dlsym(h_, "zrc4_ref_encryption"));
            name_ = "host:reference";
        } else {                                                // the C restatement (oracle/)
            mk_ = reinterpret_cast<MakeFn>(dlsym(h_, "oracle_make_sbox"));
            encL_ = reinterpret_cast<EncLongFn>(dlsym(h_, "oracle_encryption"));
            name_ = "host:oracle";
        }
        if (!mk_ || (!encI_ && !encL_)) throw std::runtime_error(lib + ": no RC4 entry points");
    }
    ~HostLibHooks() override
    {
        if (h_) dlclose(h_);
    }
    const char *name() const override { return name_; }
    uint32_t capacity() const override { return (uint32_t)(states_.size() / 258); }
    void *allocBlocks(size_t bytes) override
    {
        void *p = std::aligned_alloc(64, (bytes + 63) / 64 * 64);
        if (!p) throw std::bad_alloc();
        return p;
    }
    void freeBlocks(void *p) override { std::free(p); }
    int seed(const uint32_t *slots, uint32_t n, const std::string &key) override
    {
        for (uint32_t i = 0; i < n; ++i) mk_(st(slots[i]), key.data(), key.size());
        return ZRC4_OK;
    }
    int crypt(const Rc4Span *s, uint32_t n) override
    {
        for (uint32_t i = 0; i < n; ++i) {
            if (encI_) encI_(st(s[i].slot), s[i].data, (int)s[i].len);
            else encL_(st(s[i].slot), s[i].data, (long)s[i].len);
        }
        return ZRC4_OK;
    }

private:
    typedef void (*MakeFn)(void *, const void *, size_t);
    typedef void (*EncIntFn)(void *, void *, int);
    typedef void (*EncLongFn)(void *, void *, long);
    int *st(uint32_t slot) { return &states_[(size_t)slot * 258]; }
    void *h_ = nullptr;
    MakeFn mk_ = nullptr;
    EncIntFn encI_ = nullptr;
    EncLongFn encL_ = nullptr;
    const char *name_ = "host";
    std::vector<int> states_;
};

struct Args {
    std::string mode = "loopback";
    std::string rc4 = "device";
    std::string key = "zsummerX-rc4-stress-key";
    std::string host = "127.0.0.1";
    unsigned port = 0;
    unsigned sessions = 2;
    unsigned block = 1024;        // packet bytes incl. the 8-byte header
    unsigned depth = 1;           // packets in flight per client session
    double seconds = 3.0;
    double warmup = 0.5;
    unsigned exitAfter = 0;       // server: exit after this many sessions closed
    unsigned echoes = 0;          // client: close a session after this many echoes (0 = run by time)
    bool flashPolicy = false;
    bool plainAccepter = false;   // server: a second accepter with RC4 off (empty key, config.h:196)
    bool deviceFraming = false;   // frame receive blocks in the decrypt launch (direct device hooks)
    int device = 0;
    unsigned ring = 65536;        // keystream reservoir bytes per slot (device hooks)
};

double now()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Deterministic proto4z packet: u32 length, u16 reserve, u16 proto id, body.
void makePacket(std::vector<char> &p, unsigned block, unsigned sid, unsigned long long seq)
{
    p.resize(block);
    const uint32_t len = block;
    const uint16_t reserve = 0, proto = 30000;
    std::memcpy(&p[0], &len, 4);
    std::memcpy(&p[4], &reserve, 2);
    std::memcpy(&p[6], &proto, 2);
    for (unsigned i = 8; i < block; ++i) p[i] = (char)((seq * 131u + sid * 7u + i) & 255u);
}

struct ClientState {
    unsigned long long sent = 0, echoed = 0;
};

}  // namespace

static int run(int argc, char **argv);

int main(int argc, char **argv)
{
    try {
        return run(argc, argv);
    } catch (const std::exception &e) {
        std::fprintf(stderr, "frame_stress: %s\n", e.what());
        return 1;
    }
}

static int run(int argc, char **argv)
{
    signal(SIGPIPE, SIG_IGN);
    Args a;
    for (int i = 1; i < argc; ++i) {
        std::string k = argv[i];
        auto val = [&]() -> std::string {
            if (i + 1 >= argc) throw std::runtime_error("missing value for " + k);
            return argv[++i];
        };
        if (k == "--mode") a.mode = val();
        else if (k == "--rc4") a.rc4 = val();
        else if (k == "--key") a.key = val();
        else if (k == "--key-hex") {                       // keys with NUL bytes (std::string length counts)
            const std::string h = val();
            a.key.clear();
            for (size_t q = 0; q + 1 < h.size(); q += 2) a.key.push_back((char)std::stoul(h.substr(q, 2), nullptr, 16));
        }
        else if (k == "--host") a.host = val();
        else if (k == "--port") a.port = (unsigned)std::stoul(val());
        else if (k == "--sessions") a.sessions = (unsigned)std::stoul(val());
        else if (k == "--block") a.block = (unsigned)std::stoul(val());
        else if (k == "--depth") a.depth = (unsigned)std::stoul(val());
        else if (k == "--seconds") a.seconds = std::stod(val());
        else if (k == "--warmup") a.warmup = std::stod(val());
        else if (k == "--exit-after") a.exitAfter = (unsigned)std::stoul(val());
        else if (k == "--echoes") a.echoes = (unsigned)std::stoul(val());
        else if (k == "--flash-policy") a.flashPolicy = true;
        else if (k == "--plain-accepter") a.plainAccepter = true;
        else if (k == "--device-framing") a.deviceFraming = true;
        else if (k == "--device") a.device = std::stoi(val());
        else if (k == "--ring") a.ring = (unsigned)std::stoul(val());
        else {
            std::fprintf(stderr, "unknown option %s\n", k.c_str());
            return 2;
        }
    }
    if (a.rc4 == "off") a.key.clear();
    if (a.block < 8 || a.block > SESSION_BLOCK_SIZE) {
        std::fprintf(stderr, "--block must be in [8, %u]\n", SESSION_BLOCK_SIZE);
        return 2;
    }

    SessionManager mgr;
    const uint32_t slots = 2u * (2u * a.sessions + 1024u);   // both sides + accepted extras
    if (a.rc4 == "device") mgr.setRc4Hooks(makeDeviceRc4Hooks(a.device, slots, a.ring));
    else if (a.rc4 == "device-direct") mgr.setRc4Hooks(makeDeviceRc4Hooks(a.device, slots, 0));
    else if (a.rc4.rfind("host:", 0) == 0) mgr.setRc4Hooks(std::unique_ptr<Rc4Hooks>(new HostLibHooks(a.rc4.substr(5), slots)));
    else if (a.rc4 == "off") mgr.setRc4Hooks(makeKeylessHooks());
    else {
        std::fprintf(stderr, "--rc4 must be device, device-direct, host:<lib> or off\n");
        return 2;
    }
    mgr.setDeviceFraming(a.deviceFraming);
    mgr.start();

    unsigned long long mismatches = 0, closed = 0, linked = 0;
    std::vector<ClientState> cs;
    std::vector<std::vector<char>> lastSent;   // per client session: FIFO of packets in flight
    std::vector<std::vector<char>> expect;

    // ---- server side (CStressServerHandler)
    unsigned short port = (unsigned short)a.port;
    if (a.mode == "loopback" || a.mode == "server") {
        AccepterID aID = mgr.addAccepter("127.0.0.1", (unsigned short)a.port);
        SessionOptions &so = mgr.getAccepterOptions(aID)._sessionOptions;
        so._rc4TcpEncryption = a.key;
        so._openFlashPolicy = a.flashPolicy;
        so._maxSendListCount = 40000;                      // FrameStressMain.cpp:425
        so._onRawPacketProc = [](const TcpSessionPtr &s, const char *b, unsigned len) { s->send(b, len); };
        so._onSessionLinked = [&](const TcpSessionPtr &) { linked++; };
        so._onSessionClosed = [&](const TcpSessionPtr &) { closed++; };
        if (!mgr.openAccepter(aID)) {
            std::fprintf(stderr, "openAccepter failed\n");
            return 1;
        }
        port = mgr.getAccepterPort(aID);
        if (a.mode == "server") {
            std::printf("PORT %u\n", port);
            std::fflush(stdout);
        }
        if (a.plainAccepter) {
            // Same engine, same event loop, same hooks object: sessions of this
            // accepter have _rc4TcpEncryption == "" and must put plaintext on the
            // wire (session.cpp:313-316, 496-499, 535-538, 603-606 are skipped).
            AccepterID pID = mgr.addAccepter("127.0.0.1", 0);
            SessionOptions &po = mgr.getAccepterOptions(pID)._sessionOptions;
            po._rc4TcpEncryption.clear();
            po._maxSendListCount = 40000;
            po._onRawPacketProc = [](const TcpSessionPtr &s, const char *b, unsigned len) { s->send(b, len); };
            po._onSessionLinked = [&](const TcpSessionPtr &) { linked++; };
            po._onSessionClosed = [&](const TcpSessionPtr &) { closed++; };
            if (!mgr.openAccepter(pID)) {
                std::fprintf(stderr, "openAccepter (plain) failed\n");
                return 1;
            }
            if (a.mode == "server") {
                std::printf("PORT2 %u\n", (unsigned)mgr.getAccepterPort(pID));
                std::fflush(stdout);
            }
        }
    }

    // ---- client side (CStressClientHandler, ping-pong)
    if (a.mode == "loopback" || a.mode == "client") {
        cs.resize(a.sessions);
        expect.resize(a.sessions);
        for (unsigned i = 0; i < a.sessions; ++i) {
            SessionID cID = mgr.addConnecter(a.host, port);
            SessionOptions &o = mgr.getConnecterOptions(cID);
            o._rc4TcpEncryption = a.key;
            o._maxSendListCount = 20000;                   // FrameStressMain.cpp:402
            o._onSessionLinked = [&, i](const TcpSessionPtr &s) {
                linked++;
                std::vector<char> p;
                for (unsigned d = 0; d < a.depth; ++d) {
                    makePacket(p, a.block, i, cs[i].sent++);
                    s->send(p.data(), (unsigned)p.size());
                }
            };
            o._onRawPacketProc = [&, i](const TcpSessionPtr &s, const char *b, unsigned len) {
                ClientState &c = cs[i];
                std::vector<char> &e = expect[i];
                makePacket(e, a.block, i, c.echoed);
                if (len != a.block || std::memcmp(e.data(), b, len) != 0) mismatches++;
                c.echoed++;
                if (a.echoes && c.echoed >= a.echoes) {
                    s->close();
                    return;
                }
                std::vector<char> p;
                makePacket(p, a.block, i, c.sent++);
                s->send(p.data(), (unsigned)p.size());
            };
            o._onSessionClosed = [&](const TcpSessionPtr &) { closed++; };
            mgr.openConnecter(cID);
        }
    }

    auto echoes = [&]() {
        unsigned long long t = 0;
        for (auto &c : cs) t += c.echoed;
        return t;
    };
    const double t0 = now();
    double tw = -1, tEnd = t0 + a.warmup + a.seconds;
    unsigned long long e0 = 0, st0[STAT_SIZE] = {};
    unsigned long long iters = 0;
    for (;;) {
        mgr.runOnce(false);
        ++iters;
        const double t = now();
        if (tw < 0 && t >= t0 + a.warmup) {
            tw = t;
            e0 = echoes();
            std::memcpy(st0, mgr._statInfo, sizeof(st0));
        }
        if (t >= tEnd) break;
        if (a.mode == "server" && a.exitAfter && closed >= a.exitAfter) break;
        if (a.mode == "client" && a.echoes && mgr.sessionCount() == 0) break;
    }
    const double t1 = now();
    if (tw < 0) {
        tw = t0;
        std::memset(st0, 0, sizeof(st0));
    }
    const double dt = t1 - tw;
    const unsigned long long e1 = echoes();
    auto d = [&](int s) { return (double)(mgr._statInfo[s] - st0[s]); };
    const double calls = d(STAT_RC4_CALLS);
    std::printf(
        "{\"tool\": \"frame_stress\", \"mode\": \"%s\", \"rc4\": \"%s\", \"sessions\": %u, \"block\": %u, "
        "\"depth\": %u, \"seconds\": %.3f, \"echoes\": %llu, \"echo_per_s\": %.1f, "
        "\"rc4_calls\": %.0f, \"rc4_spans\": %.0f, \"rc4_bytes\": %.0f, \"rc4_ms\": %.3f, "
        "\"rc4_us_per_call\": %.3f, \"spans_per_call\": %.2f, \"rc4_gib_s_inside_hooks\": %.4f, "
        "\"recv_bytes\": %.0f, \"send_bytes\": %.0f, \"recv_packs\": %.0f, \"iterations\": %llu, "
        "\"device_framed\": %.0f, \"mismatches\": %llu, \"linked\": %llu, \"closed\": %llu, \"hooks\": %s}\n",
        a.mode.c_str(), mgr.rc4Hooks() ? mgr.rc4Hooks()->name() : "none", a.sessions, a.block, a.depth, dt,
        e1 - e0, (double)(e1 - e0) / dt, calls, d(STAT_RC4_SPANS), d(STAT_RC4_BYTES), d(STAT_RC4_NANOS) * 1e-6,
        calls > 0 ? d(STAT_RC4_NANOS) * 1e-3 / calls : 0.0, calls > 0 ? d(STAT_RC4_SPANS) / calls : 0.0,
        d(STAT_RC4_NANOS) > 0 ? d(STAT_RC4_BYTES) / (d(STAT_RC4_NANOS) * 1e-9) / 1073741824.0 : 0.0,
        d(STAT_RECV_BYTES), d(STAT_SEND_BYTES), d(STAT_RECV_PACKS), iters, d(STAT_RC4_FRAMED), mismatches, linked, closed,
        mgr.rc4Hooks() ? mgr.rc4Hooks()->stats().c_str() : "{}");
    std::fflush(stdout);
    return mismatches ? 3 : 0;
}
