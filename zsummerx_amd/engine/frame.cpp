// frame.cpp -- batched session engine (include/zsummerx_amd/frame.h).
//
// One runOnce() iteration (the reference runs RC4 inside each session's
// callback instead, src/frame/session.cpp:313-323 and :496-606):
//   1. epoll_wait (0 ms when sends are pending);
//   2. accept / connect completions (both RC4 streams seeded, also on accept),
//      recv into each session's _recving tail, resume partial sends;
//   3. flushHooks(): every session with a staged _sending block merges its
//      queue (session.cpp:579-601), then ONE Rc4Hooks::crypt covers every
//      fresh recv tail and every staged _sending block of the iteration;
//      encrypted blocks are written to their sockets, decrypted tails go
//      through the proto4z framing loop and dispatch (session.cpp:326-467);
//   4. closes requested during the iteration are finished.
// Per stream the keystream is consumed in wire order (a slot appears at most
// once per crypt), so the bytes on the wire equal the reference's.
#include "zsummerx_amd/frame.h"

#include <arpa/inet.h>
#include <errno.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <stdexcept>

#include "zrc4.h"

namespace zsummerx_amd {
namespace frame {

namespace {

constexpr int kMaxEvents = 5000;          // src/epoll/epoll_impl.cpp:120
constexpr int kBlockingWaitMs = 10;
constexpr unsigned kBlocksPerSlab = 256;
// Block stride: header + 20 KiB rounded to 64 B, placed so that begin[] is
// 64-byte aligned (the crypt kernel's aligned 16-B fast path).
constexpr size_t kHeader = sizeof(SessionBlock);
constexpr size_t kStride = (kHeader + SESSION_BLOCK_SIZE + 63) / 64 * 64;
constexpr size_t kLead = 64 - kHeader;   // block i starts at slab + kLead + i * kStride
static_assert(kHeader == 28, "SessionBlock header is 7 x u32 (config.h:154-164)");

const char kFlashPolicyRequest[] = "<policy-file-request/>";   // 23 bytes with the NUL
const char kFlashPolicyResponse[] =
    R"---(<cross-domain-policy><allow-access-from domain="*" to-ports="*"/></cross-domain-policy>)---";

__attribute__((format(printf, 1, 2))) void logw(const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    std::fprintf(stderr, "[zsx-frame] ");
    std::vfprintf(stderr, fmt, ap);
    std::fprintf(stderr, "\n");
    va_end(ap);
}

void setNoDelay(int fd)
{
    int one = 1;
    (void)setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

bool resolve(const std::string &host, unsigned short port, sockaddr_in &out)
{
    std::memset(&out, 0, sizeof(out));
    out.sin_family = AF_INET;
    out.sin_port = htons(port);
    if (inet_pton(AF_INET, host.c_str(), &out.sin_addr) == 1) return true;
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    if (getaddrinfo(host.c_str(), nullptr, &hints, &res) != 0 || !res) return false;
    out.sin_addr = reinterpret_cast<sockaddr_in *>(res->ai_addr)->sin_addr;
    freeaddrinfo(res);
    return true;
}

unsigned int nowSeconds() { return (unsigned int)time(nullptr); }

class KeylessHooks final : public Rc4Hooks {
public:
    const char *name() const override { return "keyless"; }
    uint32_t capacity() const override { return 0; }
    void *allocBlocks(size_t bytes) override
    {
        void *p = std::aligned_alloc(64, (bytes + 63) / 64 * 64);
        if (!p) throw std::bad_alloc();
        return p;
    }
    void freeBlocks(void *p) override { std::free(p); }
    int seed(const uint32_t *, uint32_t n, const std::string &) override
    {
        return n ? ZRC4_ERR_NO_DEVICE : ZRC4_OK;
    }
    int crypt(const Rc4Span *, uint32_t n) override { return n ? ZRC4_ERR_NO_DEVICE : ZRC4_OK; }
};

}  // namespace

// proto4z.h:704-748, restated: header length counted as LenInteger +
// ProtoInteger (6 bytes), exactly as the reference does.
RawPacketCheckResult HasRawPacket(const char *buff, unsigned int curBuffLen, unsigned int boundLen,
                                  unsigned int maxBuffLen)
{
    if (boundLen < curBuffLen || maxBuffLen < boundLen) return {BCT_CORRUPTION, curBuffLen};
    const unsigned int headLen = 4 + 2;
    if (curBuffLen < headLen) return {BCT_SHORTAGE, headLen - curBuffLen};
    unsigned int packLen;
    std::memcpy(&packLen, buff, 4);
    if (packLen < headLen) return {BCT_CORRUPTION, curBuffLen};
    if (packLen > boundLen) {
        if (packLen > maxBuffLen) return {BCT_CORRUPTION, curBuffLen};
        return {BCT_SHORTAGE, packLen - curBuffLen};
    }
    if (packLen > maxBuffLen) return {BCT_CORRUPTION, curBuffLen};
    if (packLen <= curBuffLen) return {BCT_SUCCESS, packLen};
    return {BCT_SHORTAGE, packLen - curBuffLen};
}

// ------------------------------------------------------------------ session
TcpSession::~TcpSession() { _mgr._statInfo[STAT_SESSION_DESTROYED]++; }

void TcpSession::setUserParamInteger(size_t index, unsigned long long v)
{
    if (index >= _params.size()) _params.resize(index + 1, 0);
    _params[index] = v;
}

unsigned long long TcpSession::getUserParamInteger(size_t index) const
{
    return index < _params.size() ? _params[index] : 0;
}

void TcpSession::send(const char *buf, unsigned int len)
{
    if (_status == 3 || _closing) return;
    if (!_sending) return;
    if (len > _sending->bound) {
        logw("send error: block of %u bytes exceeds the sending block bound", len);
        return;
    }
    if (len == 0) {                                          // session.cpp:479-498
        if (_status == 2 && _sending->len == 0 && !_sendque.empty()) _mgr.markDirty(*this);
        return;
    }
    if (!_sendque.empty() || _status != 2 || _sending->len != 0) {   // :503-521
        if (_sendque.size() >= _options._maxSendListCount) {
            close();
            return;
        }
        SessionBlock *sb = _mgr.CreateBlock();
        if (sb->bound < len) {
            _mgr.FreeBlock(sb);
            return;
        }
        std::memcpy(sb->begin, buf, len);
        sb->len = len;
        _sendque.push_back(sb);
        _mgr._statInfo[STAT_SEND_QUES]++;
        return;
    }
    std::memcpy(_sending->begin, buf, len);                  // :523-540, encryption deferred
    _sending->len = len;
    _sendingLen = 0;
    _sendingCrypted = false;
    _mgr._statInfo[STAT_SEND_PACKS]++;
    _mgr.markDirty(*this);
}

void TcpSession::close()
{
    if (_status == 3 || _closing) return;
    _closing = true;
    _mgr._closeList.push_back(shared_from_this());
}

// ------------------------------------------------------------------ manager
struct SessionManager::Slab {
    void *base;
};

SessionManager::SessionManager()
{
    _epfd = epoll_create1(EPOLL_CLOEXEC);
    if (_epfd < 0) throw std::runtime_error("epoll_create1 failed");
    _statInfo[STAT_STARTTIME] = (unsigned long long)time(nullptr);
}

SessionManager::~SessionManager()
{
    for (auto &kv : _sessions) {
        TcpSession &s = *kv.second;
        if (s._fd >= 0) ::close(s._fd);
        s._fd = -1;
        s._status = 3;
    }
    _sessions.clear();
    _byFd.clear();
    _recvBatch.clear();
    _dirtyList.clear();
    _sendBatch.clear();
    _closeList.clear();
    for (auto &kv : _accepters)
        if (kv.second._fd >= 0) ::close(kv.second._fd);
    if (_rc4)
        for (Slab *sl : _slabs) _rc4->freeBlocks(sl->base);
    for (Slab *sl : _slabs) delete sl;
    if (_epfd >= 0) ::close(_epfd);
}

SessionManager &SessionManager::getRef()
{
    static SessionManager m;
    return m;
}

void SessionManager::setRc4Hooks(std::unique_ptr<Rc4Hooks> h)
{
    if (!_slabs.empty()) throw std::logic_error("setRc4Hooks: blocks already allocated from the old hooks");
    _rc4 = std::move(h);
}

Rc4Hooks *SessionManager::hooks()
{
    if (!_rc4) _rc4 = makeDeviceRc4Hooks(0, 2u * 65536u);   // throws without a gfx950 device
    return _rc4.get();
}

bool SessionManager::start()
{
    hooks();
    _started = true;
    _running = true;
    return true;
}

void SessionManager::stop() { _running = false; }

bool SessionManager::run()
{
    while (_running || !_sessions.empty()) runOnce(false);
    return false;
}

SessionBlock *SessionManager::CreateBlock()
{
    if (_freeBlocks.empty()) {
        void *base = hooks()->allocBlocks(kLead + kBlocksPerSlab * kStride);
        _slabs.push_back(new Slab{base});
        char *p = static_cast<char *>(base) + kLead;
        for (unsigned i = kBlocksPerSlab; i-- > 0;) {
            SessionBlock *sb = new (p + (size_t)i * kStride) SessionBlock();
            sb->bound = SESSION_BLOCK_SIZE;
            sb->createTime = nowSeconds();
            _freeBlocks.push_back(sb);
        }
        _statInfo[STAT_EXIST_BLOCKS] += kBlocksPerSlab;
    }
    SessionBlock *sb = _freeBlocks.back();
    _freeBlocks.pop_back();
    sb->len = 0;
    sb->reused++;
    sb->timestamp = nowSeconds();
    sb->timetick = (unsigned int)std::chrono::duration_cast<std::chrono::milliseconds>(
                       std::chrono::system_clock::now().time_since_epoch()).count();
    _statInfo[STAT_FREE_BLOCKS] = _freeBlocks.size();
    return sb;
}

void SessionManager::FreeBlock(SessionBlock *sb)
{
    if (!sb) return;
    sb->len = 0;
    _freeBlocks.push_back(sb);
    _statInfo[STAT_FREE_BLOCKS] = _freeBlocks.size();
}

AccepterID SessionManager::addAccepter(const std::string &listenIP, unsigned short listenPort)
{
    const AccepterID id = ++_lastAcceptID;
    AccepterOptions &ao = _accepters[id];
    ao._aID = id;
    ao._listenIP = listenIP;
    ao._listenPort = listenPort;
    return id;
}

AccepterOptions &SessionManager::getAccepterOptions(AccepterID aID)
{
    auto it = _accepters.find(aID);
    if (it == _accepters.end()) throw std::out_of_range("unknown AccepterID");
    return it->second;
}

unsigned short SessionManager::getAccepterPort(AccepterID aID) const
{
    auto it = _accepters.find(aID);
    if (it == _accepters.end() || it->second._fd < 0) return 0;
    sockaddr_in a{};
    socklen_t l = sizeof(a);
    if (getsockname(it->second._fd, reinterpret_cast<sockaddr *>(&a), &l) != 0) return 0;
    return ntohs(a.sin_port);
}

bool SessionManager::openAccepter(AccepterID aID)
{
    AccepterOptions &ao = getAccepterOptions(aID);
    if (ao._fd >= 0) return false;
    sockaddr_in addr;
    if (!resolve(ao._listenIP.empty() ? "0.0.0.0" : ao._listenIP, ao._listenPort, addr)) return false;
    const int fd = socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
    if (fd < 0) return false;
    if (ao._setReuse) {
        int one = 1;
        (void)setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    }
    if (bind(fd, reinterpret_cast<sockaddr *>(&addr), sizeof(addr)) != 0 || listen(fd, 4096) != 0) {
        ::close(fd);
        return false;
    }
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.fd = fd;
    if (epoll_ctl(_epfd, EPOLL_CTL_ADD, fd, &ev) != 0) {
        ::close(fd);
        return false;
    }
    ao._fd = fd;
    ao._closed = false;
    _accepterByFd[fd] = aID;
    return true;
}

SessionID SessionManager::addConnecter(const std::string &remoteHost, unsigned short remotePort)
{
    const SessionID id = ++_lastConnectID;
    TcpSessionPtr s(new TcpSession(*this));
    _statInfo[STAT_SESSION_CREATED]++;
    s->_sessionID = id;
    s->_remoteIP = remoteHost;
    s->_remotePort = remotePort;
    _sessions[id] = s;
    return id;
}

SessionOptions &SessionManager::getConnecterOptions(SessionID cID)
{
    auto it = _sessions.find(cID);
    if (it == _sessions.end() || !isConnectID(cID)) throw std::out_of_range("unknown connecter SessionID");
    return it->second->_options;
}

TcpSessionPtr SessionManager::getTcpSession(SessionID sID)
{
    auto it = _sessions.find(sID);
    return it == _sessions.end() ? TcpSessionPtr() : it->second;
}

void SessionManager::seedSession(TcpSession &s)
{
    // session.cpp:110-111: both streams from the same key.
    if (s._options._rc4TcpEncryption.empty()) return;
    Rc4Hooks *h = hooks();
    if (s._slotRead == 0xFFFFFFFFu) {
        uint32_t two[2];
        for (uint32_t &v : two) {
            if (!_freeSlots.empty()) {
                v = _freeSlots.back();
                _freeSlots.pop_back();
            } else if (_nextSlot < h->capacity()) {
                v = _nextSlot++;
            } else {
                throw std::runtime_error("RC4 hooks out of stream slots");
            }
        }
        s._slotRead = two[0];
        s._slotWrite = two[1];
    }
    const uint32_t slots[2] = {s._slotRead, s._slotWrite};
    const int rc = h->seed(slots, 2, s._options._rc4TcpEncryption);
    if (rc != ZRC4_OK) throw std::runtime_error(std::string("RC4 seed failed: ") + zrc4_strerror(rc));
}

bool SessionManager::openConnecter(SessionID cID)
{
    TcpSessionPtr s = getTcpSession(cID);
    if (!s || !isConnectID(cID) || s->_status != 0) return false;
    sockaddr_in addr;
    if (!resolve(s->_remoteIP, s->_remotePort, addr)) return false;
    const int fd = socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
    if (fd < 0) return false;
    if (!s->_recving) s->_recving = CreateBlock();
    if (!s->_sending) s->_sending = CreateBlock();
    s->_recving->len = s->_sending->len = 0;
    s->_sendingLen = 0;
    seedSession(*s);                                   // session.cpp:110-111
    s->_bFirstRecvData = true;
    const int rc = ::connect(fd, reinterpret_cast<sockaddr *>(&addr), sizeof(addr));
    if (rc != 0 && errno != EINPROGRESS) {
        ::close(fd);
        return false;
    }
    s->_fd = fd;
    s->_status = 1;
    _byFd[fd] = s;
    epoll_event ev{};
    ev.events = EPOLLOUT | EPOLLIN;
    ev.data.fd = fd;
    epoll_ctl(_epfd, EPOLL_CTL_ADD, fd, &ev);
    s->_wantOut = true;
    return true;
}

bool SessionManager::attach(const TcpSessionPtr &s, int fd)
{
    // session.cpp:127-166, plus the two makeSBox calls the reference misses.
    s->_fd = fd;
    if (s->_options._setNoDelay) setNoDelay(fd);
    s->_recving = CreateBlock();
    s->_sending = CreateBlock();
    seedSession(*s);
    s->_status = 2;
    _byFd[fd] = s;
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.fd = fd;
    if (epoll_ctl(_epfd, EPOLL_CTL_ADD, fd, &ev) != 0) return false;
    _statInfo[STAT_SESSION_LINKED]++;
    if (s->_options._onSessionLinked) {
        try {
            s->_options._onSessionLinked(s);
        } catch (const std::exception &e) {
            logw("_onSessionLinked threw: %s", e.what());
        } catch (...) {
            logw("_onSessionLinked threw an unknown exception");
        }
    }
    return true;
}

void SessionManager::onAcceptable(AccepterOptions &ao)
{
    for (;;) {
        sockaddr_in peer{};
        socklen_t pl = sizeof(peer);
        const int fd = accept4(ao._fd, reinterpret_cast<sockaddr *>(&peer), &pl, SOCK_NONBLOCK | SOCK_CLOEXEC);
        if (fd < 0) {
            if (errno == EINTR) continue;
            return;                                     // EAGAIN or a transient error
        }
        if (ao._closed || ao._currentLinked >= ao._maxSessions) {   // manager.cpp:250-258
            ::close(fd);
            continue;
        }
        ao._currentLinked++;
        ao._totalAcceptCount++;
        _lastSessionID = _lastSessionID + 1 >= kMiddleSegmentValue ? 1 : _lastSessionID + 1;
        TcpSessionPtr s(new TcpSession(*this));
        _statInfo[STAT_SESSION_CREATED]++;
        s->_options = ao._sessionOptions;
        s->_acceptID = ao._aID;
        s->_sessionID = _lastSessionID;
        char ip[INET_ADDRSTRLEN] = {0};
        inet_ntop(AF_INET, &peer.sin_addr, ip, sizeof(ip));
        s->_remoteIP = ip;
        s->_remotePort = ntohs(peer.sin_port);
        _sessions[s->_sessionID] = s;
        if (!attach(s, fd)) s->close();
    }
}

void SessionManager::onConnected(const TcpSessionPtr &s)
{
    int err = 0;
    socklen_t l = sizeof(err);
    if (getsockopt(s->_fd, SOL_SOCKET, SO_ERROR, &err, &l) != 0 || err != 0) {
        s->close();                                    // no reconnects (out of scope)
        return;
    }
    s->_status = 2;
    if (s->_options._setNoDelay) setNoDelay(s->_fd);
    setWantOut(*s, false);
    if (s->_options._onSessionLinked) {
        try {
            s->_options._onSessionLinked(s);
        } catch (const std::exception &e) {
            logw("_onSessionLinked threw: %s", e.what());
        } catch (...) {
            logw("_onSessionLinked threw an unknown exception");
        }
    }
    _statInfo[STAT_SESSION_LINKED]++;
    if (!s->_sendque.empty()) markDirty(*s);           // session.cpp:205-208
}

void SessionManager::markDirty(TcpSession &s)
{
    if (s._dirty) return;
    s._dirty = true;
    _dirtyList.push_back(s.shared_from_this());
}

void SessionManager::setWantOut(TcpSession &s, bool on)
{
    if (s._wantOut == on || s._fd < 0) return;
    epoll_event ev{};
    ev.events = EPOLLIN | (on ? EPOLLOUT : 0u);
    ev.data.fd = s._fd;
    epoll_ctl(_epfd, EPOLL_CTL_MOD, s._fd, &ev);
    s._wantOut = on;
}

void SessionManager::onReadable(const TcpSessionPtr &sp)
{
    TcpSession &s = *sp;
    if (s._status != 2 || s._closing) return;
    const unsigned int before = s._recving->len;
    for (;;) {
        const unsigned int space = s._recving->bound - s._recving->len;
        if (space == 0) break;
        const ssize_t r = ::recv(s._fd, s._recving->begin + s._recving->len, space, 0);
        if (r > 0) {
            s._recving->len += (unsigned int)r;
            _statInfo[STAT_RECV_COUNT]++;
            _statInfo[STAT_RECV_BYTES] += (unsigned long long)r;
            if ((unsigned int)r < space) break;
            continue;
        }
        if (r < 0 && errno == EINTR) continue;
        if (r < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
        s.close();                                     // remote closed or socket error
        break;
    }
    const unsigned int got = s._recving->len - before;
    if (got == 0) return;
    // session.cpp:290-311: the flash-policy probe is matched on the raw
    // (still encrypted) bytes and answered through send() (so encrypted).
    if (s._bFirstRecvData) {
        s._bFirstRecvData = false;
        if (s._options._openFlashPolicy && s._acceptID != InvalidAccepterID &&
            s._recving->len == sizeof(kFlashPolicyRequest) &&
            std::memcmp(kFlashPolicyRequest, s._recving->begin, sizeof(kFlashPolicyRequest)) == 0) {
            s._recving->len = 0;
            s.send(kFlashPolicyResponse, (unsigned int)sizeof(kFlashPolicyResponse));
            return;
        }
    }
    if (s._recvFresh == 0) _recvBatch.push_back(sp);
    s._recvFresh += got;
}

void SessionManager::writeSending(const TcpSessionPtr &sp)
{
    TcpSession &s = *sp;
    while (s._sendingLen < s._sending->len) {
        const ssize_t r = ::send(s._fd, s._sending->begin + s._sendingLen, s._sending->len - s._sendingLen,
                                 MSG_NOSIGNAL);
        if (r > 0) {
            s._sendingLen += (unsigned int)r;
            _statInfo[STAT_SEND_BYTES] += (unsigned long long)r;
            continue;
        }
        if (r < 0 && errno == EINTR) continue;
        if (r < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
            setWantOut(s, true);
            return;
        }
        s.close();
        return;
    }
    // session.cpp:574-608: block done; queued blocks go out in the next flush.
    s._sending->len = 0;
    s._sendingLen = 0;
    s._sendingCrypted = false;
    setWantOut(s, false);
    if (!s._sendque.empty()) markDirty(s);
}

void SessionManager::onWritable(const TcpSessionPtr &sp)
{
    TcpSession &s = *sp;
    if (s._status != 2 || s._closing) return;
    if (s._sendingCrypted && s._sendingLen < s._sending->len) {
        _statInfo[STAT_SEND_COUNT]++;
        writeSending(sp);
    } else {
        setWantOut(s, false);
    }
}

void SessionManager::dispatchRecv(const TcpSessionPtr &sp, const Rc4Frame *fr)
{
    // session.cpp:326-467 (PT_TCP): frame and dispatch the decrypted bytes.
    // With `fr` the device already ran the check loop over this block (fused
    // into the decrypt launch): its first packets are taken from there, and
    // the host check resumes where the device list ends (it then reports the
    // same shortage / corruption the device stopped on).
    TcpSession &s = *sp;
    SessionBlock *rb = s._recving;
    unsigned int used = 0;
    uint32_t k = 0;
    const uint32_t pre = fr ? std::min(fr->npk, Rc4Frame::kMaxPackets) : 0u;
    while (!s._closing && s._status == 2) {
        RawPacketCheckResult ret;
        if (k < pre) {
            ret = RawPacketCheckResult(BCT_SUCCESS, fr->pkt[k++]);
        } else try {
            ret = s._options._onRawPacketCheck(rb->begin + used, rb->len - used, rb->bound - used, rb->bound);
        } catch (...) {
            s.close();
            return;
        }
        if (ret.first == BCT_CORRUPTION || (ret.first == BCT_SUCCESS && ret.second == 0)) {
            logw("killed socket: _onRawPacketCheck error, session %u", s._sessionID);
            s.close();
            return;
        }
        if (ret.first == BCT_SHORTAGE) break;
        _statInfo[STAT_RECV_PACKS]++;
        if (s._options._onRawPacketProc) {
            try {
                s._options._onRawPacketProc(sp, rb->begin + used, ret.second);
            } catch (const std::exception &e) {
                logw("_onRawPacketProc threw: %s", e.what());
            } catch (...) {
                logw("_onRawPacketProc threw an unknown exception");
            }
        }
        used += ret.second;
    }
    if (used > 0) {
        rb->len -= used;
        if (rb->len > 0) std::memmove(rb->begin, rb->begin + used, rb->len);
    }
}

void SessionManager::flushHooks()
{
    // Stage: merge send queues of idle sessions (session.cpp:579-601).
    for (TcpSessionPtr &sp : _dirtyList) {
        TcpSession &s = *sp;
        s._dirty = false;
        if (s._status != 2 || s._closing) continue;
        if (s._sending->len == 0 && !s._sendque.empty()) {
            do {
                SessionBlock *sb = s._sendque.front();
                s._sendque.pop_front();
                _statInfo[STAT_SEND_QUES]--;
                std::memcpy(s._sending->begin + s._sending->len, sb->begin, sb->len);
                s._sending->len += sb->len;
                FreeBlock(sb);
                _statInfo[STAT_SEND_PACKS]++;
                if (s._sendque.empty()) break;
                if (s._sending->bound - s._sending->len < s._sendque.front()->len) break;
            } while (s._options._joinSmallBlock);
            s._sendingLen = 0;
            s._sendingCrypted = false;
        }
        if (s._sending->len > 0 && !s._sendingCrypted) _sendBatch.push_back(sp);
    }
    _dirtyList.clear();

    // One crypt for the whole iteration.
    _spans.clear();
    _frames.clear();
    _recvFrame.assign(_recvBatch.size(), -1);
    const bool devFrame = _deviceFraming && _rc4 && _rc4->canFrame();
    typedef RawPacketCheckResult (*CheckFn)(const char *, unsigned int, unsigned int, unsigned int);
    for (size_t r = 0; r < _recvBatch.size(); ++r) {
        TcpSession &s = *_recvBatch[r];
        if (s._options._rc4TcpEncryption.empty() || s._recvFresh == 0 || s._recving->len == 0) continue;
        // session.cpp:315-323: the freshly received tail
        const unsigned int n = s._recvFresh < s._recving->len ? s._recvFresh : s._recving->len;
        _spans.push_back({s._slotRead, n, reinterpret_cast<uint8_t *>(s._recving->begin + s._recving->len - n)});
        if (devFrame) {
            Rc4Frame f;
            const CheckFn *fn = s._options._onRawPacketCheck.target<CheckFn>();
            if (fn && *fn == &DefaultRawPacketCheck && s._recving->bound == SESSION_BLOCK_SIZE) {
                f.block = reinterpret_cast<const uint8_t *>(s._recving->begin);
                f.len = s._recving->len;
                _recvFrame[r] = (int)_frames.size();
            }
            _frames.push_back(f);
        }
    }
    for (TcpSessionPtr &sp : _sendBatch) {
        TcpSession &s = *sp;
        if (s._options._rc4TcpEncryption.empty()) continue;
        _spans.push_back({s._slotWrite, s._sending->len, reinterpret_cast<uint8_t *>(s._sending->begin)});
        if (devFrame) _frames.emplace_back();
    }
    if (!_spans.empty()) {
        const auto t0 = std::chrono::steady_clock::now();
        const int rc = devFrame ? hooks()->cryptFrame(_spans.data(), (uint32_t)_spans.size(), _frames.data(),
                                                      SESSION_BLOCK_SIZE)
                                : hooks()->crypt(_spans.data(), (uint32_t)_spans.size());
        const auto t1 = std::chrono::steady_clock::now();
        _statInfo[STAT_RC4_CALLS]++;
        _statInfo[STAT_RC4_SPANS] += _spans.size();
        for (const Rc4Span &sp : _spans) _statInfo[STAT_RC4_BYTES] += sp.len;
        _statInfo[STAT_RC4_NANOS] +=
            (unsigned long long)std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
        if (rc != ZRC4_OK) {
            // No error channel in the reference; close the affected sessions
            // (its BCT_CORRUPTION path, session.cpp:355-361).
            logw("RC4 hooks failed: %s", zrc4_strerror(rc));
            for (TcpSessionPtr &sp : _recvBatch)
                if (!sp->_options._rc4TcpEncryption.empty()) sp->close();
            for (TcpSessionPtr &sp : _sendBatch)
                if (!sp->_options._rc4TcpEncryption.empty()) sp->close();
        }
    }

    // Write the encrypted blocks, then frame + dispatch the decrypted tails.
    for (TcpSessionPtr &sp : _sendBatch) {
        if (sp->_closing) continue;
        sp->_sendingCrypted = true;
        sp->_sendingLen = 0;
        _statInfo[STAT_SEND_COUNT]++;
        writeSending(sp);
    }
    _sendBatch.clear();
    for (size_t r = 0; r < _recvBatch.size(); ++r) {
        TcpSessionPtr &sp = _recvBatch[r];
        sp->_recvFresh = 0;
        if (sp->_closing) continue;
        const int fi = _recvFrame.empty() ? -1 : _recvFrame[r];
        if (fi >= 0) _statInfo[STAT_RC4_FRAMED]++;
        dispatchRecv(sp, fi >= 0 ? &_frames[(size_t)fi] : nullptr);
    }
    _recvBatch.clear();
}

void SessionManager::releaseSession(TcpSession &s)
{
    if (s._fd >= 0) {
        epoll_ctl(_epfd, EPOLL_CTL_DEL, s._fd, nullptr);
        ::close(s._fd);
        _byFd.erase(s._fd);
        s._fd = -1;
    }
    while (!s._sendque.empty()) {
        FreeBlock(s._sendque.front());
        s._sendque.pop_front();
        _statInfo[STAT_SEND_QUES]--;
    }
    FreeBlock(s._recving);
    FreeBlock(s._sending);
    s._recving = s._sending = nullptr;
    if (s._slotRead != 0xFFFFFFFFu) {
        _freeSlots.push_back(s._slotWrite);
        _freeSlots.push_back(s._slotRead);
        s._slotRead = s._slotWrite = 0xFFFFFFFFu;
    }
}

void SessionManager::finishCloses()
{
    while (!_closeList.empty()) {
        std::vector<TcpSessionPtr> batch;
        batch.swap(_closeList);
        for (TcpSessionPtr &sp : batch) {
            TcpSession &s = *sp;
            if (s._status == 3) continue;
            const bool wasLinked = s._status == 2;
            releaseSession(s);
            s._status = 3;
            if (s._acceptID != InvalidAccepterID) {
                auto it = _accepters.find(s._acceptID);
                if (it != _accepters.end() && it->second._currentLinked) it->second._currentLinked--;
            }
            if (wasLinked) {
                _statInfo[STAT_SESSION_CLOSED]++;
                if (s._options._onSessionClosed) {
                    try {
                        s._options._onSessionClosed(sp);
                    } catch (...) {
                        logw("_onSessionClosed threw an exception");
                    }
                }
            }
            _sessions.erase(s._sessionID);
        }
    }
}

bool SessionManager::runOnce(bool isImmediately)
{
    if (!_running && _sessions.empty()) return false;
    if (!_started) start();
    if (!_posted.empty()) {
        std::vector<std::function<void()>> p;
        p.swap(_posted);
        for (auto &h : p) h();
    }
    const bool busy = isImmediately || !_dirtyList.empty() || !_closeList.empty() || !_posted.empty();
    static thread_local epoll_event evs[kMaxEvents];
    const int n = epoll_wait(_epfd, evs, kMaxEvents, busy ? 0 : kBlockingWaitMs);
    for (int i = 0; i < n; ++i) {
        const int fd = evs[i].data.fd;
        const uint32_t e = evs[i].events;
        auto ai = _accepterByFd.find(fd);
        if (ai != _accepterByFd.end()) {
            auto it = _accepters.find(ai->second);
            if (it != _accepters.end() && !it->second._closed) onAcceptable(it->second);
            continue;
        }
        auto si = _byFd.find(fd);
        if (si == _byFd.end()) continue;
        TcpSessionPtr s = si->second;
        if (s->_status == 1) {
            if (e & (EPOLLOUT | EPOLLERR | EPOLLHUP)) onConnected(s);
            if (s->_status != 2) continue;
        }
        if (e & (EPOLLIN | EPOLLERR | EPOLLHUP)) onReadable(s);
        if (e & EPOLLOUT) onWritable(s);
    }
    flushHooks();
    finishCloses();
    return true;
}

void SessionManager::sendSessionData(SessionID sID, const char *orgData, unsigned int orgDataLen)
{
    TcpSessionPtr s = getTcpSession(sID);
    if (s) s->send(orgData, orgDataLen);
}

void SessionManager::kickSession(SessionID sID)
{
    TcpSessionPtr s = getTcpSession(sID);
    if (s) {
        if (s->_status == 0) {            // never opened: just forget it
            _sessions.erase(sID);
            return;
        }
        s->close();
    }
}

void SessionManager::kickClientSession(AccepterID aID)
{
    for (auto &kv : _sessions)
        if (isSessionID(kv.first) && (aID == InvalidAccepterID || kv.second->_acceptID == aID)) kv.second->close();
}

void SessionManager::kickConnect(SessionID cID)
{
    std::vector<SessionID> fresh;
    for (auto &kv : _sessions) {
        if (!isConnectID(kv.first) || (cID != InvalidSessionID && kv.first != cID)) continue;
        if (kv.second->_status == 0) fresh.push_back(kv.first);
        else kv.second->close();
    }
    for (SessionID id : fresh) _sessions.erase(id);
}

void SessionManager::stopAccept(AccepterID aID)
{
    for (auto &kv : _accepters) {
        if (aID != InvalidAccepterID && kv.first != aID) continue;
        AccepterOptions &ao = kv.second;
        ao._closed = true;
        if (ao._fd >= 0) {
            epoll_ctl(_epfd, EPOLL_CTL_DEL, ao._fd, nullptr);
            ::close(ao._fd);
            _accepterByFd.erase(ao._fd);
            ao._fd = -1;
        }
    }
}

}  // namespace frame

std::unique_ptr<Rc4Hooks> makeKeylessHooks() { return std::unique_ptr<Rc4Hooks>(new frame::KeylessHooks()); }

}  // namespace zsummerx_amd
