// zsummerx_amd/frame.h -- batched session engine: the caller side of the RC4
// path, with the reference frame API's names and
// argument meaning so a zsummerX user finds what they know:
//
//   SessionOptions / AccepterOptions      include/zsummerX/frame/config.h:187-227
//   SessionBlock, SESSION_BLOCK_SIZE      include/zsummerX/frame/config.h:100, 154-164
//   BLOCK_CHECK_TYPE, StatType            include/zsummerX/frame/config.h:108-146
//   TcpSession::send / close              src/frame/session.cpp:470-545, 234-266
//   SessionManager (start/run/runOnce, addAccepter/openAccepter,
//     addConnecter/openConnecter, sendSessionData, kickSession, ...)
//                                         include/zsummerX/frame/manager.h:78-186
//   DefaultRawPacketCheck -> HasRawPacket include/zsummerX/frame/manager.h:53-57,
//                                         depends/proto4z/proto4z.h:704-748
//
// What differs (by design, MI355X-first):
//   * RC4 is not called per session.  One runOnce() iteration gathers every
//     recv tail (session.cpp:313-323) and every outgoing _sending block
//     (:496-499, :535-538, :603-606) and crypts them with ONE Rc4Hooks::crypt
//     call -- one gfx950 launch over pinned SessionBlocks.  Each stream's
//     keystream order is the wire byte order, so the bytes on the wire are
//     exactly the reference's (wire-compatible with RC4Encryption peers).
//   * Both RC4 streams are seeded on connect AND on accept.  The reference
//     never seeds accepted sessions (session.cpp:127-166),
//     which leaves their S-box indeterminate; this is a documented divergence.
//   * One event loop on Linux epoll, single-threaded like the reference's
//     (manager.h:98-110).  Timers, reconnects, HTTP, whitelists, UDP and the
//     Lua/log layers are out of scope.
#pragma once

#include <cstdint>
#include <deque>
#include <functional>
#include <memory>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "rc4_hooks.h"

namespace zsummerx_amd {
namespace frame {

using SessionID = unsigned int;
using AccepterID = unsigned int;
const SessionID InvalidSessionID = (SessionID)-1;
const AccepterID InvalidAccepterID = (AccepterID)-1;

// Session ids below the middle value are accepted sessions, above are
// connecters (config.h:90-96).
const unsigned int kMiddleSegmentValue = 300u * 1000u * 1000u;
inline bool isSessionID(unsigned int id) { return id != InvalidSessionID && id < kMiddleSegmentValue; }
inline bool isConnectID(unsigned int id) { return id != InvalidSessionID && id >= kMiddleSegmentValue; }

const unsigned int SESSION_BLOCK_SIZE = 20 * 1024;   // config.h:100

enum BLOCK_CHECK_TYPE {
    BCT_SUCCESS = 0,     // a whole packet: second = its length
    BCT_SHORTAGE = 1,    // need more bytes
    BCT_CORRUPTION = 2,  // close the session
};

enum StatType {
    STAT_STARTTIME,
    STAT_SESSION_CREATED,
    STAT_SESSION_DESTROYED,
    STAT_SESSION_LINKED,
    STAT_SESSION_CLOSED,
    STAT_FREE_BLOCKS,
    STAT_EXIST_BLOCKS,
    STAT_SEND_COUNT,
    STAT_SEND_PACKS,
    STAT_SEND_BYTES,
    STAT_SEND_QUES,
    STAT_RECV_COUNT,
    STAT_RECV_PACKS,
    STAT_RECV_BYTES,
    // engine-only counters (batched hooks)
    STAT_RC4_CALLS,      // Rc4Hooks::crypt calls (one per busy iteration)
    STAT_RC4_SPANS,      // spans crypted (reference: one encryption() call each)
    STAT_RC4_BYTES,      // bytes crypted
    STAT_RC4_NANOS,      // wall time inside Rc4Hooks::crypt
    STAT_RC4_FRAMED,     // receive blocks framed on the device (setDeviceFraming)
    STAT_SIZE,
};

// config.h:154-164: same header layout (7 x u32, then the bytes).
struct SessionBlock {
    unsigned int type = 0;
    unsigned int createTime = 0;
    unsigned int reused = 0;
    unsigned int timestamp = 0;
    unsigned int timetick = 0;
    unsigned int bound = 0;
    unsigned int len = 0;
    char begin[0];
};

class TcpSession;
using TcpSessionPtr = std::shared_ptr<TcpSession>;
using RawPacketCheckResult = std::pair<BLOCK_CHECK_TYPE, unsigned int>;
using OnBlockCheck = std::function<RawPacketCheckResult(const char * /*begin*/, unsigned int /*len*/,
                                                        unsigned int /*bound*/, unsigned int /*blockLimit*/)>;
using OnBlockDispatch = std::function<void(const TcpSessionPtr &, const char * /*begin*/, unsigned int /*len*/)>;
using OnSessionEvent = std::function<void(const TcpSessionPtr &)>;

// proto4z framing (depends/proto4z/proto4z.h:704-748): header = u32 packet
// length (header included) + u16 reserve + u16 proto id, little-endian.
RawPacketCheckResult HasRawPacket(const char *buff, unsigned int curBuffLen, unsigned int boundLen,
                                  unsigned int maxBuffLen);
inline RawPacketCheckResult DefaultRawPacketCheck(const char *begin, unsigned int len, unsigned int bound,
                                                  unsigned int blockLimit)
{
    return HasRawPacket(begin, len, bound, blockLimit);
}

struct SessionOptions {                       // config.h:187-212 (TCP subset)
    std::string _rc4TcpEncryption;            // empty = RC4 off
    bool _openFlashPolicy = false;
    bool _setNoDelay = true;
    bool _joinSmallBlock = true;              // merge queued blocks into one send
    unsigned int _maxSendListCount = 600;
    OnBlockCheck _onRawPacketCheck = DefaultRawPacketCheck;
    OnBlockDispatch _onRawPacketProc;
    OnSessionEvent _onSessionClosed;
    OnSessionEvent _onSessionLinked;
};

struct AccepterOptions {                      // config.h:214-227 (subset)
    AccepterID _aID = InvalidAccepterID;
    std::string _listenIP;
    unsigned short _listenPort = 0;
    bool _setReuse = true;
    unsigned int _maxSessions = 5000;
    unsigned long long _totalAcceptCount = 0;
    unsigned long long _currentLinked = 0;
    bool _closed = false;
    SessionOptions _sessionOptions;
    int _fd = -1;
};

class SessionManager;

class TcpSession : public std::enable_shared_from_this<TcpSession> {
public:
    ~TcpSession();
    SessionID getSessionID() const { return _sessionID; }
    AccepterID getAcceptID() const { return _acceptID; }
    const std::string &getRemoteIP() const { return _remoteIP; }
    unsigned short getRemotePort() const { return _remotePort; }
    SessionOptions &getOptions() { return _options; }
    bool isInvalidSession() const { return _status != 2; }

    // session.cpp:470-545.  Queues or stages the bytes; encryption and the
    // socket write happen in the iteration's batched flush, in call order.
    void send(const char *buf, unsigned int len);
    void close();

    void setUserParamInteger(size_t index, unsigned long long v);
    unsigned long long getUserParamInteger(size_t index) const;

    // RC4 stream slots (_rc4StateRead / _rc4StateWrite, session.h:115-116).
    uint32_t readSlot() const { return _slotRead; }
    uint32_t writeSlot() const { return _slotWrite; }

private:
    friend class SessionManager;
    explicit TcpSession(SessionManager &m) : _mgr(m) {}

    SessionManager &_mgr;
    SessionOptions _options;
    SessionID _sessionID = InvalidSessionID;
    AccepterID _acceptID = InvalidAccepterID;
    std::string _remoteIP;
    unsigned short _remotePort = 0;
    int _fd = -1;
    int _status = 0;          // 0 new, 1 connecting, 2 linked, 3 closed (session.h)
    SessionBlock *_recving = nullptr;
    SessionBlock *_sending = nullptr;
    unsigned int _sendingLen = 0;     // bytes of _sending already written
    bool _sendingCrypted = false;     // _sending holds wire bytes
    std::deque<SessionBlock *> _sendque;
    uint32_t _slotRead = 0xFFFFFFFFu, _slotWrite = 0xFFFFFFFFu;
    bool _bFirstRecvData = true;
    unsigned int _recvFresh = 0;      // bytes received this iteration (to decrypt)
    bool _dirty = false;              // in the manager's send-flush list
    bool _wantOut = false;            // EPOLLOUT registered
    bool _closing = false;            // close requested (deferred to iteration end)
    std::vector<unsigned long long> _params;
};

class SessionManager {
public:
    // One engine per event-loop thread.  getRef() is the process-wide one, as
    // in the reference (manager.h:78-84); other instances may be made freely.
    SessionManager();
    ~SessionManager();
    static SessionManager &getRef();

    // Install the RC4 hooks before start() (default: makeDeviceRc4Hooks(0,
    // 2 * maxSessions) the first time a session with a key needs one).
    void setRc4Hooks(std::unique_ptr<Rc4Hooks> hooks);
    Rc4Hooks *rc4Hooks() const { return _rc4.get(); }
    // Frame decrypted receive blocks on the device, fused into the decrypt
    // launch (Rc4Hooks::cryptFrame), for sessions whose
    // _onRawPacketCheck is the default proto4z check.  Needs hooks with
    // canFrame() (the direct device hooks); otherwise framing stays on the host.
    void setDeviceFraming(bool on) { _deviceFraming = on; }

    bool start();
    void stop();
    bool run();
    bool runOnce(bool isImmediately = false);
    bool isRunning() const { return _running; }
    void post(std::function<void()> h) { _posted.push_back(std::move(h)); }

    AccepterID addAccepter(const std::string &listenIP, unsigned short listenPort);
    AccepterOptions &getAccepterOptions(AccepterID aID);
    bool openAccepter(AccepterID aID);
    unsigned short getAccepterPort(AccepterID aID) const;   // bound port (listenPort 0 -> ephemeral)

    SessionID addConnecter(const std::string &remoteHost, unsigned short remotePort);
    SessionOptions &getConnecterOptions(SessionID cID);
    bool openConnecter(SessionID cID);
    TcpSessionPtr getTcpSession(SessionID sID);

    void sendSessionData(SessionID sID, const char *orgData, unsigned int orgDataLen);
    void kickSession(SessionID sID);
    void kickClientSession(AccepterID aID = InvalidAccepterID);
    void kickConnect(SessionID cID = InvalidSessionID);
    void stopAccept(AccepterID aID = InvalidAccepterID);

    unsigned long long getStatInfo(int stat) const { return _statInfo[stat]; }
    unsigned long long _statInfo[STAT_SIZE] = {};
    size_t sessionCount() const { return _sessions.size(); }

    // Block pool (manager.cpp:290-332) over Rc4Hooks::allocBlocks memory
    // (pinned host memory for the device hooks).
    SessionBlock *CreateBlock();
    void FreeBlock(SessionBlock *sb);

private:
    friend class TcpSession;
    struct Slab;

    Rc4Hooks *hooks();
    bool attach(const TcpSessionPtr &s, int fd);
    void seedSession(TcpSession &s);
    void releaseSession(TcpSession &s);
    void onAcceptable(AccepterOptions &ao);
    void onConnected(const TcpSessionPtr &s);
    void onReadable(const TcpSessionPtr &s);
    void onWritable(const TcpSessionPtr &s);
    void markDirty(TcpSession &s);
    void writeSending(const TcpSessionPtr &s);
    void setWantOut(TcpSession &s, bool on);
    void dispatchRecv(const TcpSessionPtr &s, const Rc4Frame *fr = nullptr);
    void flushHooks();
    void finishCloses();

    std::unique_ptr<Rc4Hooks> _rc4;
    int _epfd = -1;
    bool _running = true;
    bool _started = false;
    AccepterID _lastAcceptID = 0;
    SessionID _lastSessionID = 0;
    SessionID _lastConnectID = kMiddleSegmentValue;
    std::unordered_map<SessionID, TcpSessionPtr> _sessions;
    std::unordered_map<AccepterID, AccepterOptions> _accepters;
    std::unordered_map<int, TcpSessionPtr> _byFd;
    std::unordered_map<int, AccepterID> _accepterByFd;

    // per-iteration batches
    std::vector<TcpSessionPtr> _recvBatch;    // sessions with fresh bytes to decrypt
    std::vector<TcpSessionPtr> _dirtyList;    // sessions with _sending to encrypt
    std::vector<TcpSessionPtr> _sendBatch;    // sessions whose _sending is in this crypt
    std::vector<TcpSessionPtr> _closeList;
    std::vector<Rc4Span> _spans;
    std::vector<Rc4Frame> _frames;            // parallel to _spans when framing on the device
    std::vector<int> _recvFrame;              // _recvBatch[i] -> its frame in _frames, or -1
    bool _deviceFraming = false;
    std::vector<std::function<void()>> _posted;

    // slots and blocks
    std::vector<uint32_t> _freeSlots;
    uint32_t _nextSlot = 0;
    std::vector<Slab *> _slabs;
    std::vector<SessionBlock *> _freeBlocks;
};

}  // namespace frame
}  // namespace zsummerx_amd
