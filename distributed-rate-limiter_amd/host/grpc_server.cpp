// grpc_server.cpp -- the native gRPC front end (include/rl_grpc.h).
//
// Threads: `io_threads` event loops, each with its own SO_REUSEPORT listener,
// epoll set, connections (one nghttp2 server session each) and RPC table.  A
// complete request is decoded and submitted to the coalescer right away
// (Coalescer::Submit with the loop as completion tag); the coalescer's
// notification hook queues the ticket to that loop (eventfd), which collects
// the results with a non-blocking Wait and writes the response.  So an event
// loop never blocks on the GPU, and the coalescer batches the RPCs of all
// loops and connections into the same launches.
#include "../../include/rl_grpc.h"

#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <string.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <memory>
#include <mutex>
#include <queue>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/rl_keyhash.h"
#include "../csrc/rl_semantics.h"
#include "coalescer.hpp"
#include "h2.hpp"

namespace {

constexpr int GRPC_OK = 0, GRPC_CANCELLED = 1, GRPC_INVALID_ARGUMENT = 3, GRPC_DEADLINE_EXCEEDED = 4,
              GRPC_NOT_FOUND = 5, GRPC_UNIMPLEMENTED = 12, GRPC_INTERNAL = 13, GRPC_UNAVAILABLE = 14;
const char* const ERR_INVALID_N = "invalid n: must be greater than 0";   // errors.go:16

int64_t realtime_ns() {
    timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    return (int64_t)ts.tv_sec * 1000000000LL + ts.tv_nsec;
}

// ---------------------------------------------------------------------------
// protobuf wire format (the proto3 subset of api/proto/*.proto)
// ---------------------------------------------------------------------------
struct Pb {
    const uint8_t* p;
    const uint8_t* e;
    bool ok = true;
    bool more() const { return ok && p < e; }
    uint64_t varint() {
        uint64_t v = 0;
        for (int s = 0; s < 70; s += 7) {
            if (p >= e) { ok = false; return 0; }
            const uint8_t b = *p++;
            v |= (uint64_t)(b & 0x7f) << s;
            if (!(b & 0x80)) return v;
        }
        ok = false;
        return 0;
    }
    std::string_view bytes() {
        const uint64_t n = varint();
        if (!ok || n > (uint64_t)(e - p)) { ok = false; return {}; }
        std::string_view v((const char*)p, (size_t)n);
        p += n;
        return v;
    }
    void skip(uint32_t wt) {
        if (wt == 0) (void)varint();
        else if (wt == 2) (void)bytes();
        else if (wt == 1 && e - p >= 8) p += 8;
        else if (wt == 5 && e - p >= 4) p += 4;
        else ok = false;
    }
};

void put_varint(std::string& o, uint64_t v) {
    while (v >= 0x80) {
        o.push_back((char)(v | 0x80));
        v >>= 7;
    }
    o.push_back((char)v);
}
void put_int(std::string& o, uint32_t field, int64_t v) {   // int64 / bool / enum, omitted when 0
    if (!v) return;
    put_varint(o, (uint64_t)field << 3);
    put_varint(o, (uint64_t)v);
}
void put_bytes(std::string& o, uint32_t field, std::string_view v) {
    if (v.empty()) return;
    put_varint(o, ((uint64_t)field << 3) | 2);
    put_varint(o, v.size());
    o.append(v.data(), v.size());
}

// AllowRequest / AllowNRequest / ResetRequest: limiter = 1, key = 2, n = 3
struct ReqMsg {
    std::string_view limiter, key;
    int64_t n = 0;
};
bool parse_req(std::string_view m, ReqMsg* r) {
    Pb pb{(const uint8_t*)m.data(), (const uint8_t*)m.data() + m.size()};
    while (pb.more()) {
        const uint64_t tag = pb.varint();
        const uint32_t f = (uint32_t)(tag >> 3), wt = (uint32_t)(tag & 7);
        if (f == 1 && wt == 2) r->limiter = pb.bytes();
        else if (f == 2 && wt == 2) r->key = pb.bytes();
        else if (f == 3 && wt == 0) r->n = (int64_t)pb.varint();
        else pb.skip(wt);
    }
    return pb.ok;
}

struct Result {
    bool allowed = false;
    int64_t limit = 0, remaining = 0, retry = 0, reset = 0;
    std::string error;
};
void put_allow_response(std::string& o, const Result& r) {
    put_int(o, 1, r.allowed ? 1 : 0);
    put_int(o, 2, r.limit);
    put_int(o, 3, r.remaining);
    put_int(o, 4, r.retry);
    put_int(o, 5, r.reset);
    put_bytes(o, 6, r.error);
}

// Python's repr() of a str as the handlers format it: 'name' (no quote inside)
std::string py_repr(std::string_view s) {
    const bool sq = s.find('\'') != std::string_view::npos && s.find('"') == std::string_view::npos;
    const char q = sq ? '"' : '\'';
    std::string o(1, q);
    for (char c : s) {
        if (c == '\\' || c == q) o.push_back('\\');
        o.push_back(c);
    }
    o.push_back(q);
    return o;
}

// grpc-message is percent-encoded (gRPC over HTTP/2 spec)
std::string pct(std::string_view s) {
    static const char* hx = "0123456789ABCDEF";
    std::string o;
    for (unsigned char c : s) {
        if (c >= 0x20 && c <= 0x7e && c != '%') o.push_back((char)c);
        else {
            o.push_back('%');
            o.push_back(hx[c >> 4]);
            o.push_back(hx[c & 15]);
        }
    }
    return o;
}

// grpc-timeout: 1-8 digits and a unit (H M S m u n)
int64_t parse_timeout(std::string_view v) {
    if (v.size() < 2 || v.size() > 9) return -1;
    int64_t x = 0;
    for (size_t i = 0; i + 1 < v.size(); i++) {
        if (v[i] < '0' || v[i] > '9') return -1;
        x = x * 10 + (v[i] - '0');
    }
    int64_t unit;
    switch (v.back()) {
        case 'H': unit = 3600 * 1000000000LL; break;
        case 'M': unit = 60 * 1000000000LL; break;
        case 'S': unit = 1000000000LL; break;
        case 'm': unit = 1000000LL; break;
        case 'u': unit = 1000LL; break;
        case 'n': unit = 1; break;
        default: return -1;
    }
    // the header comes from the network: saturate instead of overflowing
    // (99999999H is ~1.1e4 years of nanoseconds)
    return x > INT64_MAX / unit ? INT64_MAX : x * unit;
}

// a timeout this long (~100 years, e.g. grpc-go's 2562047H maximum) is no deadline
constexpr int64_t NO_DEADLINE_NS = 100LL * 365 * 24 * 3600 * 1000000000LL;

// ---------------------------------------------------------------------------
// server state
// ---------------------------------------------------------------------------
struct Limiter {
    std::string name, prefix;
    uint32_t cfg = 0;
    int32_t alg = 0;
    bool fail_open = false;
    int64_t limit = 0, window = 0;
    rl::CfgDev hc{};
    // Result.ResetAt of the fail-open path (tokenbucket.go:101-109,
    // slidingwindow.go:84-92, fixedwindow.go:80-88)
    int64_t fail_open_reset_at(int64_t t) const {
        if (alg == rl::ALG_TOKEN_BUCKET) return rl::tb_reset_at((double)t / 1e9, hc);
        return rl::wadd(rl::wmul(rl::window_start(t, hc), rl::NS_PER_S), hc.window);
    }
};

struct Io;
struct Conn;

enum Kind : uint8_t { K_ALLOW, K_BATCH, K_RESET };

struct Stream {
    int32_t id = 0;
    std::string path, body, resp;
    size_t resp_off = 0;
    int64_t timeout_ns = -1;
    uint64_t ticket = 0;
    bool pending = false;      // an RPC waits for the coalescer
};

struct BatchItem {
    const Limiter* lim;
    int64_t n;
    int err;                   // 0: submitted; 1: unknown limiter; 2: invalid n
    std::string name;          // the unknown limiter's name
};

struct Rpc {
    Conn* conn;
    int32_t sid;
    Kind kind;
    int64_t t;                 // time.Now() of the RPC
    int64_t deadline;          // coalescer clock, 0 = none
    const Limiter* lim = nullptr;
    std::vector<BatchItem> items;
    size_t m = 0;              // requests submitted
};

struct Server;

struct Conn {
    Io* io;
    int fd;
    nghttp2_session* ss = nullptr;
    std::unordered_map<int32_t, std::unique_ptr<Stream>> streams;
    std::string wbuf;
    size_t woff = 0;
    bool dirty = false, closing = false, want_out = false;
};

struct Io {
    Server* srv;
    int idx = 0;
    int ep = -1, lfd = -1, efd = -1;
    std::thread th;
    std::mutex mu;
    std::vector<uint64_t> done;             // tickets completed (from the coalescer)
    std::unordered_map<uint64_t, Rpc> rpcs; // by ticket
    std::vector<Conn*> conns;
    std::vector<Conn*> dirty;
    using Dl = std::pair<int64_t, uint64_t>;
    std::priority_queue<Dl, std::vector<Dl>, std::greater<Dl>> deadlines;
};

struct Server {
    rlc::Coalescer* co = nullptr;
    std::vector<Limiter> lims;
    std::unordered_map<std::string, const Limiter*> by_name;
    bool isolate = false;
    int64_t clock_start = 0, clock_step = 0;
    std::atomic<int64_t> clock_k{0};
    std::atomic<bool> serving{true}, stopping{false};
    int64_t stop_deadline = 0;
    int port = 0;
    std::vector<std::unique_ptr<Io>> ios;
    nghttp2_session_callbacks* cbs = nullptr;
    std::atomic<uint64_t> n_conn{0}, n_rpc{0}, n_dec{0}, n_err{0}, n_cancel{0};

    int64_t now() {
        if (!clock_step) return realtime_ns();
        return clock_start + (clock_k.fetch_add(1) + 1) * clock_step;
    }
    const Limiter* find(std::string_view name) const {
        auto it = by_name.find(std::string(name));
        return it == by_name.end() ? nullptr : it->second;
    }
    uint64_t key_id(const Limiter* l, std::string_view key) const {
        uint64_t off[2] = {0, key.size()}, id = 0;
        const uint32_t cfg = l->cfg;
        (void)rl_hash_keys_host(1, (const uint8_t*)key.data(), key.size(), off, 0, isolate ? &cfg : nullptr,
                                l->prefix.data(), l->prefix.size(), &id);
        return id;
    }
};

// the coalescer's completion hook: hand the ticket to its event loop
void on_done(void*, uint64_t ticket, void* tag) {
    Io* io = static_cast<Io*>(tag);
    bool wake;
    {
        std::lock_guard<std::mutex> g(io->mu);
        wake = io->done.empty();
        io->done.push_back(ticket);
    }
    if (wake) {
        const uint64_t one = 1;
        ssize_t r = write(io->efd, &one, 8);
        (void)r;
    }
}

// ---------------------------------------------------------------------------
// responses
// ---------------------------------------------------------------------------
ssize_t read_body(nghttp2_session* ss, int32_t sid, uint8_t* buf, size_t len, uint32_t* flags,
                  nghttp2_data_source* src, void*) {
    Stream* st = static_cast<Stream*>(src->ptr);
    const size_t n = std::min(len, st->resp.size() - st->resp_off);
    memcpy(buf, st->resp.data() + st->resp_off, n);
    st->resp_off += n;
    if (st->resp_off == st->resp.size()) {
        *flags |= h2::DATA_FLAG_EOF | h2::DATA_FLAG_NO_END_STREAM;
        const nghttp2_nv tr[] = {h2::nv("grpc-status", 11, "0", 1)};
        nghttp2_submit_trailer(ss, sid, tr, 1);
    }
    return (ssize_t)n;
}

void mark_dirty(Conn* c) {
    if (!c->dirty) {
        c->dirty = true;
        c->io->dirty.push_back(c);
    }
}

// a gRPC message (uncompressed) as the response body
void respond_ok(Conn* c, Stream* st, const std::string& msg) {
    st->resp.clear();
    st->resp.push_back(0);
    const uint32_t n = (uint32_t)msg.size();
    const char len[4] = {(char)(n >> 24), (char)(n >> 16), (char)(n >> 8), (char)n};
    st->resp.append(len, 4);
    st->resp += msg;
    st->resp_off = 0;
    const nghttp2_nv hd[] = {h2::nv(":status", 7, "200", 3), h2::nv("content-type", 12, "application/grpc", 16)};
    nghttp2_data_provider prd;
    prd.source.ptr = st;
    prd.read_callback = read_body;
    nghttp2_submit_response(c->ss, st->id, hd, 2, &prd);
    c->io->srv->n_rpc++;
    mark_dirty(c);
}

// trailers-only response with a non-OK status
void respond_err(Conn* c, Stream* st, int code, std::string_view msg) {
    char cs[12];
    const int cl = snprintf(cs, sizeof cs, "%d", code);
    const std::string m = pct(msg);
    const nghttp2_nv hd[] = {h2::nv(":status", 7, "200", 3), h2::nv("content-type", 12, "application/grpc", 16),
                             h2::nv("grpc-status", 11, cs, (size_t)cl), h2::nv("grpc-message", 12, m.data(), m.size())};
    nghttp2_submit_response(c->ss, st->id, hd, m.empty() ? 3 : 4, nullptr);
    c->io->srv->n_rpc++;
    c->io->srv->n_err++;
    mark_dirty(c);
}

// AllowResponse of one decision, or the error branch (python/rl_server.py _result)
struct Outcome {
    Result r;
    int code = GRPC_OK;        // fail-closed: the status of the error branch
};
Outcome decide_outcome(const Limiter* lim, int64_t t, int rc, uint8_t dec, int64_t rem, int64_t retry,
                       int64_t reset) {
    Outcome o;
    if (rc == RL_OK && (dec == RL_ALLOWED || dec == RL_DENIED)) {
        o.r.allowed = dec == RL_ALLOWED;
        o.r.limit = lim->limit;
        o.r.remaining = rem;
        o.r.retry = retry;
        o.r.reset = reset;
        return o;
    }
    std::string err;
    int code = GRPC_UNAVAILABLE;
    if (rc == RL_EDEADLINE) {
        err = "context deadline exceeded";
        code = GRPC_DEADLINE_EXCEEDED;
    } else if (rc == RL_ECANCELED) {
        err = "context canceled";
        code = GRPC_CANCELLED;
    } else if (rc != RL_OK) {
        err = "engine status " + std::to_string(rc);
    } else {
        err = "script error (INCRBY overflow)";
    }
    if (lim->fail_open) {   // FailOpen: {Allowed, Limit, 0, 0, ResetAt}, no error
        o.r.allowed = true;
        o.r.limit = lim->limit;
        o.r.reset = lim->fail_open_reset_at(t);
        return o;
    }
    o.code = code;
    o.r.error = "failed to check rate limit: " + err;
    return o;
}

// ---------------------------------------------------------------------------
// request dispatch
// ---------------------------------------------------------------------------
void finish_rpc(Io* io, uint64_t ticket, Rpc& rpc, int rc, const uint8_t* dec, const int64_t* rem,
                const int64_t* retry, const int64_t* reset) {
    Conn* c = rpc.conn;
    auto it = c->streams.find(rpc.sid);
    if (it == c->streams.end()) return;   // the client went away
    Stream* st = it->second.get();
    st->pending = false;
    std::string msg;
    if (rpc.kind == K_RESET) {
        if (rc != RL_OK) respond_err(c, st, GRPC_UNAVAILABLE, "failed to reset rate limit: engine status " + std::to_string(rc));
        else respond_ok(c, st, msg);
        return;
    }
    if (rpc.kind == K_ALLOW) {
        const Outcome o = decide_outcome(rpc.lim, rpc.t, rc, dec ? dec[0] : 0, rem ? rem[0] : 0, retry ? retry[0] : 0,
                                         reset ? reset[0] : 0);
        if (o.code != GRPC_OK) return respond_err(c, st, o.code, o.r.error);
        put_allow_response(msg, o.r);
        return respond_ok(c, st, msg);
    }
    size_t j = 0;
    std::string one;
    for (const BatchItem& b : rpc.items) {
        Result r;
        if (b.err == 1) r.error = "unknown limiter " + py_repr(b.name);
        else if (b.err == 2) r.error = ERR_INVALID_N;
        else {
            r = decide_outcome(b.lim, rpc.t, rc, dec ? dec[j] : 0, rem ? rem[j] : 0, retry ? retry[j] : 0,
                               reset ? reset[j] : 0).r;
            j++;
        }
        one.clear();
        put_allow_response(one, r);
        put_varint(msg, (1u << 3) | 2);
        put_varint(msg, one.size());
        msg += one;
    }
    (void)ticket;
    respond_ok(c, st, msg);
}

// collect a completed (or expired) ticket: Wait without blocking
void collect(Io* io, uint64_t ticket) {
    auto it = io->rpcs.find(ticket);
    if (it == io->rpcs.end()) return;   // already collected (a deadline, a cancel)
    Rpc& rpc = it->second;
    const size_t m = rpc.kind == K_RESET ? 0 : rpc.m;
    std::vector<uint8_t> dec(m);
    std::vector<int64_t> rem(m), retry(m), reset(m);
    const int rc = io->srv->co->Wait(ticket, 0, dec.data(), rem.data(), retry.data(), reset.data());
    if (rc == RL_ETIMEOUT) return;      // not done yet (a spurious wake)
    finish_rpc(io, ticket, rpc, rc, dec.data(), rem.data(), retry.data(), reset.data());
    io->rpcs.erase(it);
}

void submit_rpc(Io* io, Conn* c, Stream* st, Rpc&& rpc, size_t m, const uint64_t* key, const int64_t* ts,
                const int64_t* n, const uint32_t* cfg) {
    Server* s = io->srv;
    rpc.deadline = st->timeout_ns >= 0 && st->timeout_ns < NO_DEADLINE_NS
                       ? std::max<int64_t>(1, rlc::steady_ns() + st->timeout_ns)   // no overflow below the bound
                       : 0;
    uint64_t ticket = 0;
    int rc;
    if (rpc.kind == K_RESET) rc = s->co->SubmitOp(rlc::OP_RESET, key[0], ts[0], cfg[0], 0, 0, 0, &ticket, io);
    else rc = s->co->Submit(m, key, ts, n, cfg, &ticket, rpc.deadline, io);
    s->n_dec += m;
    if (rc != RL_OK) {   // queue full / closed: the error branch at once
        finish_rpc(io, 0, rpc, rc, nullptr, nullptr, nullptr, nullptr);
        return;
    }
    st->pending = true;
    st->ticket = ticket;
    if (rpc.deadline) io->deadlines.push({rpc.deadline, ticket});
    io->rpcs.emplace(ticket, std::move(rpc));
}

void dispatch(Conn* c, Stream* st) {
    Io* io = c->io;
    Server* s = io->srv;
    const std::string& b = st->body;
    if (b.size() < 5 || b[0] != 0) return respond_err(c, st, GRPC_INTERNAL, "malformed or compressed message");
    const uint32_t len = ((uint32_t)(uint8_t)b[1] << 24) | ((uint32_t)(uint8_t)b[2] << 16) |
                         ((uint32_t)(uint8_t)b[3] << 8) | (uint32_t)(uint8_t)b[4];
    if (len != b.size() - 5) return respond_err(c, st, GRPC_INTERNAL, "message length mismatch");
    const std::string_view msg(b.data() + 5, len);
    static const std::string svc = "/ratelimiter.v1.RateLimiter/";
    const std::string& p = st->path;
    if (p == "/grpc.health.v1.Health/Check") {
        ReqMsg r;   // HealthCheckRequest.service = 1
        if (!parse_req(msg, &r)) return respond_err(c, st, GRPC_INTERNAL, "bad HealthCheckRequest");
        const int status = (r.limiter.empty() || r.limiter == "ratelimiter.v1.RateLimiter") ? (s->serving ? 1 : 2) : 3;
        std::string out;
        put_int(out, 1, status);
        return respond_ok(c, st, out);
    }
    if (p.compare(0, svc.size(), svc) != 0) return respond_err(c, st, GRPC_UNIMPLEMENTED, "unknown service");
    const std::string m = p.substr(svc.size());
    if (m == "Allow" || m == "AllowN" || m == "Reset") {
        ReqMsg r;
        if (!parse_req(msg, &r)) return respond_err(c, st, GRPC_INTERNAL, "bad request message");
        const Limiter* lim = s->find(r.limiter);
        if (!lim) return respond_err(c, st, GRPC_NOT_FOUND, "unknown limiter " + py_repr(r.limiter));
        if (m == "Allow") r.n = 1;
        if (m == "AllowN" && r.n <= 0) return respond_err(c, st, GRPC_INVALID_ARGUMENT, ERR_INVALID_N);
        const int64_t t = s->now();
        const uint64_t id = s->key_id(lim, r.key);
        const size_t mm = m == "Reset" ? 0 : 1;
        Rpc rpc{c, st->id, m == "Reset" ? K_RESET : K_ALLOW, t, 0, lim, {}, mm};
        const int64_t n = r.n;
        const uint32_t cfg = lim->cfg;
        return submit_rpc(io, c, st, std::move(rpc), mm, &id, &t, &n, &cfg);
    }
    if (m == "AllowBatch") {
        Rpc rpc{c, st->id, K_BATCH, s->now(), 0, nullptr, {}, 0};
        std::vector<uint64_t> key;
        std::vector<int64_t> ts, n;
        std::vector<uint32_t> cfg;
        Pb pb{(const uint8_t*)msg.data(), (const uint8_t*)msg.data() + msg.size()};
        while (pb.more()) {
            const uint64_t tag = pb.varint();
            if ((tag >> 3) != 1 || (tag & 7) != 2) {
                pb.skip((uint32_t)(tag & 7));
                continue;
            }
            ReqMsg r;
            if (!parse_req(pb.bytes(), &r) || !pb.ok) return respond_err(c, st, GRPC_INTERNAL, "bad AllowBatchRequest");
            BatchItem it{s->find(r.limiter), r.n, 0, {}};
            if (!it.lim) {
                it.err = 1;
                it.name = std::string(r.limiter);
            } else if (r.n <= 0) {
                it.err = 2;
            } else {
                key.push_back(s->key_id(it.lim, r.key));
                ts.push_back(rpc.t);
                n.push_back(r.n);
                cfg.push_back(it.lim->cfg);
            }
            rpc.items.push_back(std::move(it));
        }
        if (!pb.ok) return respond_err(c, st, GRPC_INTERNAL, "bad AllowBatchRequest");
        rpc.m = key.size();
        if (rpc.m == 0) return finish_rpc(io, 0, rpc, RL_OK, nullptr, nullptr, nullptr, nullptr);
        const size_t mm = rpc.m;
        return submit_rpc(io, c, st, std::move(rpc), mm, key.data(), ts.data(), n.data(), cfg.data());
    }
    respond_err(c, st, GRPC_UNIMPLEMENTED, "unknown method " + m);
}

// ---------------------------------------------------------------------------
// nghttp2 callbacks
// ---------------------------------------------------------------------------
Stream* get_stream(Conn* c, int32_t sid) {
    auto it = c->streams.find(sid);
    return it == c->streams.end() ? nullptr : it->second.get();
}

int cb_begin_headers(nghttp2_session*, const nghttp2_frame* f, void* u) {
    Conn* c = static_cast<Conn*>(u);
    if (f->hd.type != h2::HEADERS) return 0;
    auto& p = c->streams[f->hd.stream_id];
    if (!p) {
        p.reset(new Stream());
        p->id = f->hd.stream_id;
    }
    return 0;
}

int cb_header(nghttp2_session*, const nghttp2_frame* f, const uint8_t* name, size_t nl, const uint8_t* value, size_t vl,
              uint8_t, void* u) {
    Stream* st = get_stream(static_cast<Conn*>(u), f->hd.stream_id);
    if (!st) return 0;
    const std::string_view n((const char*)name, nl), v((const char*)value, vl);
    if (n == ":path") st->path.assign(v);
    else if (n == "grpc-timeout") st->timeout_ns = parse_timeout(v);
    return 0;
}

int cb_data(nghttp2_session*, uint8_t, int32_t sid, const uint8_t* data, size_t len, void* u) {
    Stream* st = get_stream(static_cast<Conn*>(u), sid);
    if (st) {
        if (st->body.size() + len > (4u << 20)) return h2::ERR_CALLBACK_FAILURE;   // 4 MiB per request
        st->body.append((const char*)data, len);
    }
    return 0;
}

int cb_frame(nghttp2_session*, const nghttp2_frame* f, void* u) {
    Conn* c = static_cast<Conn*>(u);
    if ((f->hd.type == h2::HEADERS || f->hd.type == h2::DATA) && (f->hd.flags & h2::FLAG_END_STREAM)) {
        Stream* st = get_stream(c, f->hd.stream_id);
        if (st) dispatch(c, st);
    }
    return 0;
}

int cb_close(nghttp2_session*, int32_t sid, uint32_t, void* u) {
    Conn* c = static_cast<Conn*>(u);
    auto it = c->streams.find(sid);
    if (it == c->streams.end()) return 0;
    Stream* st = it->second.get();
    if (st->pending) {
        // the client reset the stream (its deadline, ctx cancel): cancel the
        // submission -- dropped unapplied if not launched -- and release it
        Io* io = c->io;
        io->srv->co->Cancel(st->ticket);
        auto r = io->rpcs.find(st->ticket);
        if (r != io->rpcs.end()) {
            (void)io->srv->co->Wait(st->ticket, 0, nullptr, nullptr, nullptr, nullptr);
            io->rpcs.erase(r);
        }
        io->srv->n_cancel++;
    }
    c->streams.erase(it);
    return 0;
}

// ---------------------------------------------------------------------------
// event loop
// ---------------------------------------------------------------------------
void close_conn(Io* io, Conn* c) {
    // streams still waiting: cancel and release their submissions
    for (auto& kv : c->streams) {
        Stream* st = kv.second.get();
        if (!st->pending) continue;
        io->srv->co->Cancel(st->ticket);
        auto r = io->rpcs.find(st->ticket);
        if (r != io->rpcs.end()) {
            (void)io->srv->co->Wait(st->ticket, 0, nullptr, nullptr, nullptr, nullptr);
            io->rpcs.erase(r);
        }
    }
    c->streams.clear();
    epoll_ctl(io->ep, EPOLL_CTL_DEL, c->fd, nullptr);
    close(c->fd);
    nghttp2_session_del(c->ss);
    io->conns.erase(std::remove(io->conns.begin(), io->conns.end(), c), io->conns.end());
    io->dirty.erase(std::remove(io->dirty.begin(), io->dirty.end(), c), io->dirty.end());
    delete c;
}

// serialize what the session wants to send and write it; false: close
bool flush(Io* io, Conn* c) {
    c->dirty = false;
    for (;;) {
        const uint8_t* d = nullptr;
        const ssize_t n = nghttp2_session_mem_send(c->ss, &d);
        if (n < 0) return false;
        if (n == 0) break;
        c->wbuf.append((const char*)d, (size_t)n);
    }
    while (c->woff < c->wbuf.size()) {
        const ssize_t w = ::send(c->fd, c->wbuf.data() + c->woff, c->wbuf.size() - c->woff, MSG_NOSIGNAL);
        if (w < 0) {
            if (errno == EINTR) continue;
            if (errno == EAGAIN || errno == EWOULDBLOCK) break;
            return false;
        }
        c->woff += (size_t)w;
    }
    if (c->woff == c->wbuf.size()) {
        c->wbuf.clear();
        c->woff = 0;
    } else if (c->woff > (1u << 20)) {
        c->wbuf.erase(0, c->woff);
        c->woff = 0;
    }
    const bool out = !c->wbuf.empty();
    if (out != c->want_out) {
        epoll_event ev{};
        ev.events = EPOLLIN | (out ? EPOLLOUT : 0u);
        ev.data.ptr = c;
        epoll_ctl(io->ep, EPOLL_CTL_MOD, c->fd, &ev);
        c->want_out = out;
    }
    if (!nghttp2_session_want_read(c->ss) && !nghttp2_session_want_write(c->ss) && c->wbuf.empty()) return false;
    return true;
}

void accept_all(Io* io) {
    Server* s = io->srv;
    for (;;) {
        const int fd = accept4(io->lfd, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
        if (fd < 0) return;
        if (s->stopping) {
            close(fd);
            continue;
        }
        const int one = 1;
        setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
        Conn* c = new Conn{io, fd};
        nghttp2_session_server_new(&c->ss, s->cbs, c);
        const nghttp2_settings_entry iv[] = {{h2::SETTINGS_MAX_CONCURRENT_STREAMS, 4096},
                                             {h2::SETTINGS_INITIAL_WINDOW_SIZE, 1 << 20}};
        nghttp2_submit_settings(c->ss, 0, iv, 2);
        nghttp2_session_set_local_window_size(c->ss, 0, 0, 16 << 20);
        epoll_event ev{};
        ev.events = EPOLLIN;
        ev.data.ptr = c;
        epoll_ctl(io->ep, EPOLL_CTL_ADD, fd, &ev);
        io->conns.push_back(c);
        s->n_conn++;
        mark_dirty(c);
    }
}

bool read_conn(Conn* c) {
    uint8_t buf[65536];
    for (;;) {
        const ssize_t r = ::recv(c->fd, buf, sizeof buf, 0);
        if (r == 0) return false;
        if (r < 0) {
            if (errno == EINTR) continue;
            return errno == EAGAIN || errno == EWOULDBLOCK;
        }
        if (nghttp2_session_mem_recv(c->ss, buf, (size_t)r) < 0) return false;
        mark_dirty(c);
        if ((size_t)r < sizeof buf) return true;
    }
}

char tag_listen, tag_event;   // epoll data of the listener and the eventfd

void loop(Io* io) {
    Server* s = io->srv;
    epoll_event evs[256];
    for (;;) {
        int timeout_ms = 50;
        if (!io->deadlines.empty()) {
            const int64_t d = io->deadlines.top().first - rlc::steady_ns();
            timeout_ms = d <= 0 ? 0 : (int)std::min<int64_t>(50, (d + 999999) / 1000000);
        }
        const int n = epoll_wait(io->ep, evs, 256, timeout_ms);
        for (int i = 0; i < n; i++) {
            void* p = evs[i].data.ptr;
            if (p == &tag_listen) {
                accept_all(io);
            } else if (p == &tag_event) {
                uint64_t v;
                ssize_t r = read(io->efd, &v, 8);
                (void)r;
                std::vector<uint64_t> done;
                {
                    std::lock_guard<std::mutex> g(io->mu);
                    done.swap(io->done);
                }
                for (uint64_t t : done) collect(io, t);
            } else {
                Conn* c = static_cast<Conn*>(p);
                bool ok = true;
                if (evs[i].events & (EPOLLIN | EPOLLHUP | EPOLLERR)) ok = read_conn(c);
                if (ok && (evs[i].events & EPOLLOUT)) mark_dirty(c);
                if (!ok) close_conn(io, c);
            }
        }
        // server-side deadlines of RPCs still queued (or running)
        const int64_t now = rlc::steady_ns();
        while (!io->deadlines.empty() && io->deadlines.top().first <= now) {
            const uint64_t t = io->deadlines.top().second;
            io->deadlines.pop();
            collect(io, t);
        }
        std::vector<Conn*> dirty;
        dirty.swap(io->dirty);
        for (Conn* c : dirty)
            if (!flush(io, c)) close_conn(io, c);
        if (s->stopping) {
            if (io->lfd >= 0) {
                epoll_ctl(io->ep, EPOLL_CTL_DEL, io->lfd, nullptr);
                close(io->lfd);
                io->lfd = -1;
            }
            if (io->rpcs.empty() || rlc::steady_ns() >= s->stop_deadline) {
                for (Conn* c : std::vector<Conn*>(io->conns)) {
                    nghttp2_submit_goaway(c->ss, 0, nghttp2_session_get_last_proc_stream_id(c->ss), 0, nullptr, 0);
                    (void)flush(io, c);
                    close_conn(io, c);
                }
                return;
            }
        }
    }
}

int listen_on(const char* host, int port, int* bound) {
    const int fd = socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
    if (fd < 0) return -1;
    const int one = 1;
    setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    setsockopt(fd, SOL_SOCKET, SO_REUSEPORT, &one, sizeof one);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)port);
    if (inet_pton(AF_INET, host, &a.sin_addr) != 1 || bind(fd, (sockaddr*)&a, sizeof a) != 0 || listen(fd, 1024) != 0) {
        close(fd);
        return -1;
    }
    socklen_t sl = sizeof a;
    getsockname(fd, (sockaddr*)&a, &sl);
    *bound = ntohs(a.sin_port);
    return fd;
}

}  // namespace

struct rl_grpc_server {
    Server s;
};

extern "C" int rl_grpc_server_start(rl_coalescer* c, const rl_grpc_limiter* limiters, size_t n_limiters,
                                    const rl_grpc_opts* opts, rl_grpc_server** out) {
    rlc::Coalescer* co = rlc::unwrap(c);
    if (!co || !out || (n_limiters && !limiters) || (opts && opts->struct_size != sizeof(rl_grpc_opts)))
        return RL_EINVAL;
    rl_grpc_opts o{};
    if (opts) o = *opts;
    const int nio = o.io_threads ? (int)o.io_threads : 4;
    if (nio > 64) return RL_EINVAL;
    auto* g = new rl_grpc_server();
    Server& s = g->s;
    s.co = co;
    s.isolate = o.isolate != 0;
    s.clock_start = o.clock_start_ns;
    s.clock_step = o.clock_step_ns;
    s.lims.reserve(n_limiters);
    for (size_t i = 0; i < n_limiters; i++) {
        const rl_grpc_limiter& l = limiters[i];
        if (l.struct_size != sizeof(rl_grpc_limiter) || !l.name) {
            delete g;
            return RL_EINVAL;
        }
        Limiter L;
        L.name = l.name;
        L.prefix = (l.prefix && *l.prefix) ? l.prefix : "ratelimit";   // WithDefaults (config.go:62-64)
        L.cfg = l.cfg_id;
        L.alg = l.algorithm;
        L.fail_open = l.fail_open != 0;
        L.limit = l.limit;
        L.window = l.window_ns;
        L.hc = rl::make_cfg(l.algorithm, l.limit, l.window_ns);
        s.lims.push_back(L);
    }
    for (const Limiter& L : s.lims) s.by_name[L.name] = &L;
    nghttp2_session_callbacks_new(&s.cbs);
    nghttp2_session_callbacks_set_on_begin_headers_callback(s.cbs, cb_begin_headers);
    nghttp2_session_callbacks_set_on_header_callback(s.cbs, cb_header);
    nghttp2_session_callbacks_set_on_data_chunk_recv_callback(s.cbs, cb_data);
    nghttp2_session_callbacks_set_on_frame_recv_callback(s.cbs, cb_frame);
    nghttp2_session_callbacks_set_on_stream_close_callback(s.cbs, cb_close);
    co->SetNotify(on_done, &s);
    const char* host = o.host ? o.host : "127.0.0.1";
    int port = o.port;
    for (int i = 0; i < nio; i++) {
        auto io = std::make_unique<Io>();
        io->srv = &s;
        io->idx = i;
        io->lfd = listen_on(host, port, &port);
        io->ep = epoll_create1(EPOLL_CLOEXEC);
        io->efd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
        bool ok = io->lfd >= 0 && io->ep >= 0 && io->efd >= 0;
        if (ok) {
            epoll_event ev{};
            ev.events = EPOLLIN;
            ev.data.ptr = &tag_listen;
            ok = epoll_ctl(io->ep, EPOLL_CTL_ADD, io->lfd, &ev) == 0;
            ev.data.ptr = &tag_event;
            ok = ok && epoll_ctl(io->ep, EPOLL_CTL_ADD, io->efd, &ev) == 0;
        }
        s.ios.push_back(std::move(io));
        if (!ok) {
            co->SetNotify(nullptr, nullptr);
            for (auto& x : s.ios)
                for (int fd : {x->lfd, x->ep, x->efd})
                    if (fd >= 0) close(fd);
            nghttp2_session_callbacks_del(s.cbs);
            delete g;
            return RL_EDEVICE;
        }
    }
    s.port = port;
    for (auto& io : s.ios) {
        Io* p = io.get();
        p->th = std::thread([p] { loop(p); });
    }
    *out = g;
    return RL_OK;
}

extern "C" int rl_grpc_server_port(rl_grpc_server* g) { return g ? g->s.port : RL_EINVAL; }

extern "C" int rl_grpc_server_shutdown(rl_grpc_server* g, int64_t grace_ns) {
    if (!g) return RL_EINVAL;
    Server& s = g->s;
    if (s.stopping.exchange(true)) return RL_OK;
    s.serving = false;
    s.stop_deadline = rlc::steady_ns() + (grace_ns > 0 ? grace_ns : 0);
    for (auto& io : s.ios) {
        const uint64_t one = 1;
        ssize_t r = write(io->efd, &one, 8);
        (void)r;
    }
    for (auto& io : s.ios)
        if (io->th.joinable()) io->th.join();
    return RL_OK;
}

extern "C" int rl_grpc_server_destroy(rl_grpc_server* g) {
    if (!g) return RL_EINVAL;
    rl_grpc_server_shutdown(g, 0);
    Server& s = g->s;
    s.co->SetNotify(nullptr, nullptr);
    for (auto& io : s.ios) {
        close(io->ep);
        close(io->efd);
        if (io->lfd >= 0) close(io->lfd);
    }
    if (s.cbs) nghttp2_session_callbacks_del(s.cbs);
    delete g;
    return RL_OK;
}

extern "C" int rl_grpc_server_get_stats(rl_grpc_server* g, rl_grpc_stats* out) {
    if (!g || !out || out->struct_size < 8) return RL_EINVAL;
    Server& s = g->s;
    rl_grpc_stats r{};
    r.struct_size = sizeof r;
    r.connections = s.n_conn;
    r.rpcs = s.n_rpc;
    r.decisions = s.n_dec;
    r.errors = s.n_err;
    r.cancelled = s.n_cancel;
    const uint32_t n = (uint32_t)std::min<size_t>(out->struct_size, sizeof r);   // bytes filled in
    r.struct_size = n;
    memcpy(out, &r, n);
    return RL_OK;
}
