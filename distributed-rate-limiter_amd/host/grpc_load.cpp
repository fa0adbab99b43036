// grpc_load.cpp -- open-loop gRPC load generator for BASELINE configs[4]
// (the rate limiter service, api/proto/ratelimiter.proto).
//
// T threads, each with C HTTP/2 connections (nghttp2 client sessions, h2c),
// send Allow (or AllowBatch of B AllowN requests) RPCs on a fixed schedule:
// thread k sends its i-th RPC at t0 + (i * T + k) / rate, whatever the
// server's progress (open loop).  A request's latency runs from its SCHEDULED
// send time to its response trailers, so time spent queued in this client
// counts too (no coordinated omission).  Keys "user:<id>", id = a seeded
// permutation of Zipf(s) ranks over `keys` users (s = 1.5: the top key draws
// 38 % of requests).
//
//   rl_grpc_load --addr 127.0.0.1:8080 --rate 35000 --seconds 3 [--batch 1]
//                [--threads 4] [--conns 2] [--limiter default] [--zipf 1.5]
//                [--keys 1000000] [--timeout-ms 0] [--warmup 0.3] [--seed 1]
// prints one JSON line.
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <sys/timerfd.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <memory>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "h2.hpp"

namespace {

int64_t mono_ns() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (int64_t)ts.tv_sec * 1000000000LL + ts.tv_nsec;
}

struct Args {
    std::string host = "127.0.0.1", limiter = "default";
    int port = 8080, threads = 4, conns = 2, batch = 1;
    double rate = 10000, seconds = 3, zipf = 1.5, warmup = 0.3;
    int64_t keys = 1000000, timeout_ms = 0;
    uint64_t seed = 1;
};

// Zipf(s) over [0, n) by inverse CDF, ranks mapped through a seeded permutation
struct Zipf {
    std::vector<double> cdf;
    std::vector<uint32_t> perm;
    Zipf(int64_t n, double s, uint64_t seed) : cdf(n), perm(n) {
        double acc = 0;
        for (int64_t i = 0; i < n; i++) cdf[i] = acc += std::pow((double)(i + 1), -s);
        for (auto& c : cdf) c /= acc;
        for (int64_t i = 0; i < n; i++) perm[i] = (uint32_t)i;
        std::mt19937_64 g(seed ^ 0x5eedULL);
        std::shuffle(perm.begin(), perm.end(), g);
    }
    uint32_t sample(double u) const {
        const size_t r = (size_t)(std::lower_bound(cdf.begin(), cdf.end(), u) - cdf.begin());
        return perm[std::min(r, cdf.size() - 1)];
    }
};

void put_varint(std::string& o, uint64_t v) {
    while (v >= 0x80) {
        o.push_back((char)(v | 0x80));
        v >>= 7;
    }
    o.push_back((char)v);
}
void put_str(std::string& o, uint32_t f, const std::string& s) {
    put_varint(o, (f << 3) | 2);
    put_varint(o, s.size());
    o += s;
}

struct Call {
    int64_t sched = 0;
    std::string body;
    size_t off = 0;
    int status = -1;          // grpc-status of the trailers
    bool measured = false;
};

struct Thread;
struct Conn {
    Thread* th = nullptr;
    int fd = -1;
    nghttp2_session* ss = nullptr;
    std::string wbuf;
    size_t woff = 0;
    bool want_out = false, dead = false;
};

struct Thread {
    const Args* a = nullptr;
    const Zipf* z = nullptr;
    int idx = 0;
    int ep = -1, tfd = -1;
    std::vector<Conn*> conns;
    std::vector<double> lat_us;
    uint64_t sent = 0, ok = 0, errors = 0, outstanding = 0, send_fail = 0;
    int64_t t0 = 0, t_warm = 0, t_end = 0;
    std::string path, authority, timeout;
    std::mt19937_64 rng;
};

ssize_t read_body(nghttp2_session*, int32_t, uint8_t* buf, size_t len, uint32_t* flags, nghttp2_data_source* src,
                  void*) {
    Call* c = static_cast<Call*>(src->ptr);
    const size_t n = std::min(len, c->body.size() - c->off);
    memcpy(buf, c->body.data() + c->off, n);
    c->off += n;
    if (c->off == c->body.size()) *flags |= h2::DATA_FLAG_EOF;
    return (ssize_t)n;
}

int cb_header(nghttp2_session* ss, const nghttp2_frame* f, const uint8_t* name, size_t nl, const uint8_t* value,
              size_t vl, uint8_t, void*) {
    if (nl == 11 && memcmp(name, "grpc-status", 11) == 0) {
        Call* c = static_cast<Call*>(nghttp2_session_get_stream_user_data(ss, f->hd.stream_id));
        if (c) c->status = atoi(std::string((const char*)value, vl).c_str());
    }
    return 0;
}

int cb_close(nghttp2_session* ss, int32_t sid, uint32_t, void* u) {
    Thread* t = static_cast<Conn*>(u)->th;
    Call* c = static_cast<Call*>(nghttp2_session_get_stream_user_data(ss, sid));
    if (!c) return 0;
    const int64_t now = mono_ns();
    t->outstanding--;
    if (c->status == 0) {
        t->ok++;
        if (c->measured) t->lat_us.push_back((double)(now - c->sched) / 1e3);
    } else {
        t->errors++;
    }
    delete c;
    return 0;
}

bool flush(Thread* t, Conn* c) {
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
    }
    const bool out = !c->wbuf.empty();
    if (out != c->want_out) {
        epoll_event ev{};
        ev.events = EPOLLIN | (out ? EPOLLOUT : 0u);
        ev.data.ptr = c;
        epoll_ctl(t->ep, EPOLL_CTL_MOD, c->fd, &ev);
        c->want_out = out;
    }
    return true;
}

bool read_conn(Conn* c) {
    uint8_t buf[65536];
    for (;;) {
        const ssize_t r = ::recv(c->fd, buf, sizeof buf, 0);
        if (r == 0) return false;
        if (r < 0) return errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR;
        if (nghttp2_session_mem_recv(c->ss, buf, (size_t)r) < 0) return false;
        if ((size_t)r < sizeof buf) return true;
    }
}

int connect_to(const Args& a) {
    const int fd = socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
    if (fd < 0) return -1;
    sockaddr_in sa{};
    sa.sin_family = AF_INET;
    sa.sin_port = htons((uint16_t)a.port);
    if (inet_pton(AF_INET, a.host.c_str(), &sa.sin_addr) != 1 || connect(fd, (sockaddr*)&sa, sizeof sa) != 0) {
        close(fd);
        return -1;
    }
    const int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    fcntl(fd, F_SETFL, fcntl(fd, F_GETFL) | O_NONBLOCK);
    return fd;
}

// one RPC: the request message and its HEADERS
void send_call(Thread* t, Conn* c, int64_t sched) {
    const Args& a = *t->a;
    Call* call = new Call();
    call->sched = sched;
    call->measured = sched >= t->t_warm;
    std::string msg, one;
    std::uniform_real_distribution<double> U(0.0, 1.0);
    if (a.batch <= 1) {
        put_str(msg, 1, a.limiter);
        put_str(msg, 2, "user:" + std::to_string(t->z->sample(U(t->rng))));
    } else {
        for (int i = 0; i < a.batch; i++) {
            one.clear();
            put_str(one, 1, a.limiter);
            put_str(one, 2, "user:" + std::to_string(t->z->sample(U(t->rng))));
            put_varint(one, 3 << 3);
            put_varint(one, 1);
            put_str(msg, 1, one);
        }
    }
    call->body.push_back(0);
    const uint32_t n = (uint32_t)msg.size();
    const char len[4] = {(char)(n >> 24), (char)(n >> 16), (char)(n >> 8), (char)n};
    call->body.append(len, 4);
    call->body += msg;
    nghttp2_nv hd[7] = {h2::nv(":method", 7, "POST", 4), h2::nv(":scheme", 7, "http", 4),
                        h2::nv(":path", 5, t->path.data(), t->path.size()),
                        h2::nv(":authority", 10, t->authority.data(), t->authority.size()),
                        h2::nv("content-type", 12, "application/grpc", 16), h2::nv("te", 2, "trailers", 8),
                        h2::nv("grpc-timeout", 12, t->timeout.data(), t->timeout.size())};
    nghttp2_data_provider prd;
    prd.source.ptr = call;
    prd.read_callback = read_body;
    const int32_t sid = nghttp2_submit_request(c->ss, nullptr, hd, t->timeout.empty() ? 6 : 7, &prd, call);
    if (sid < 0) {
        delete call;
        t->send_fail++;
        return;
    }
    t->sent++;
    t->outstanding++;
}

void run_thread(Thread* t, nghttp2_session_callbacks* cbs) {
    const Args& a = *t->a;
    t->ep = epoll_create1(EPOLL_CLOEXEC);
    t->tfd = timerfd_create(CLOCK_MONOTONIC, TFD_NONBLOCK | TFD_CLOEXEC);
    {
        epoll_event ev{};
        ev.events = EPOLLIN;
        ev.data.ptr = nullptr;
        epoll_ctl(t->ep, EPOLL_CTL_ADD, t->tfd, &ev);
    }
    for (int i = 0; i < a.conns; i++) {
        Conn* c = new Conn();
        c->th = t;
        c->fd = connect_to(a);
        if (c->fd < 0) {
            delete c;
            continue;
        }
        nghttp2_session_client_new(&c->ss, cbs, c);
        const nghttp2_settings_entry iv[] = {{h2::SETTINGS_MAX_CONCURRENT_STREAMS, 4096},
                                             {h2::SETTINGS_INITIAL_WINDOW_SIZE, 1 << 20}};
        nghttp2_submit_settings(c->ss, 0, iv, 2);
        nghttp2_session_set_local_window_size(c->ss, 0, 0, 16 << 20);
        epoll_event ev{};
        ev.events = EPOLLIN;
        ev.data.ptr = c;
        epoll_ctl(t->ep, EPOLL_CTL_ADD, c->fd, &ev);
        t->conns.push_back(c);
        flush(t, c);
    }
    if (t->conns.empty()) return;
    const double period = (double)a.threads / a.rate * 1e9;        // ns between this thread's RPCs
    const int64_t first = t->t0 + (int64_t)((double)t->idx / a.rate * 1e9);
    uint64_t i = 0;
    size_t rr = 0;
    epoll_event evs[64];
    const int64_t drain_until = t->t_end + 5000000000LL;
    for (;;) {
        const int64_t now = mono_ns();
        // every RPC whose scheduled time has come
        while (true) {
            const int64_t sched = first + (int64_t)((double)i * period);
            if (sched > now || sched >= t->t_end) break;
            Conn* c = t->conns[rr++ % t->conns.size()];
            if (!c->dead) send_call(t, c, sched);
            i++;
        }
        for (Conn* c : t->conns)
            if (!c->dead && !flush(t, c)) c->dead = true;
        const int64_t next = first + (int64_t)((double)i * period);
        if (now >= t->t_end && t->outstanding == 0) break;
        if (now >= drain_until) break;
        itimerspec its{};
        const int64_t when = next < t->t_end ? next : now + 1000000;
        its.it_value.tv_sec = when / 1000000000LL;
        its.it_value.tv_nsec = when % 1000000000LL;
        timerfd_settime(t->tfd, TFD_TIMER_ABSTIME, &its, nullptr);
        const int n = epoll_wait(t->ep, evs, 64, 100);
        for (int k = 0; k < n; k++) {
            if (!evs[k].data.ptr) {
                uint64_t x;
                ssize_t r = read(t->tfd, &x, 8);
                (void)r;
                continue;
            }
            Conn* c = static_cast<Conn*>(evs[k].data.ptr);
            if (c->dead) continue;
            if (!read_conn(c)) c->dead = true;
        }
    }
    for (Conn* c : t->conns) {
        close(c->fd);
        nghttp2_session_del(c->ss);
        delete c;
    }
    close(t->tfd);
    close(t->ep);
}

double pct(std::vector<double>& v, double p) {
    if (v.empty()) return NAN;
    const size_t k = std::min(v.size() - 1, (size_t)std::floor(p / 100.0 * (double)(v.size() - 1) + 0.5));
    std::nth_element(v.begin(), v.begin() + k, v.end());
    return v[k];
}

}  // namespace

int main(int argc, char** argv) {
    Args a;
    for (int i = 1; i + 1 < argc; i += 2) {
        const std::string k = argv[i], v = argv[i + 1];
        if (k == "--addr") {
            const size_t c = v.rfind(':');
            a.host = v.substr(0, c);
            a.port = atoi(v.c_str() + c + 1);
        } else if (k == "--rate") a.rate = atof(v.c_str());
        else if (k == "--seconds") a.seconds = atof(v.c_str());
        else if (k == "--threads") a.threads = atoi(v.c_str());
        else if (k == "--conns") a.conns = atoi(v.c_str());
        else if (k == "--batch") a.batch = atoi(v.c_str());
        else if (k == "--limiter") a.limiter = v;
        else if (k == "--zipf") a.zipf = atof(v.c_str());
        else if (k == "--keys") a.keys = atoll(v.c_str());
        else if (k == "--timeout-ms") a.timeout_ms = atoll(v.c_str());
        else if (k == "--warmup") a.warmup = atof(v.c_str());
        else if (k == "--seed") a.seed = strtoull(v.c_str(), nullptr, 10);
        else {
            fprintf(stderr, "unknown option %s\n", k.c_str());
            return 2;
        }
    }
    if (a.threads < 1 || a.conns < 1 || a.rate <= 0 || a.seconds <= 0) return 2;
    const Zipf z(a.keys, a.zipf, a.seed);
    nghttp2_session_callbacks* cbs;
    nghttp2_session_callbacks_new(&cbs);
    nghttp2_session_callbacks_set_on_header_callback(cbs, cb_header);
    nghttp2_session_callbacks_set_on_stream_close_callback(cbs, cb_close);
    std::vector<std::unique_ptr<Thread>> ts;
    const int64_t t0 = mono_ns() + 200000000LL;   // connections set up first
    for (int k = 0; k < a.threads; k++) {
        auto t = std::make_unique<Thread>();
        t->a = &a;
        t->z = &z;
        t->idx = k;
        t->t0 = t0;
        t->t_warm = t0 + (int64_t)(a.warmup * 1e9);
        t->t_end = t0 + (int64_t)((a.warmup + a.seconds) * 1e9);
        t->path = a.batch <= 1 ? "/ratelimiter.v1.RateLimiter/Allow" : "/ratelimiter.v1.RateLimiter/AllowBatch";
        t->authority = a.host + ":" + std::to_string(a.port);
        if (a.timeout_ms > 0) t->timeout = std::to_string(a.timeout_ms) + "m";
        t->rng.seed(a.seed * 1000003ULL + (uint64_t)k);
        ts.push_back(std::move(t));
    }
    std::vector<std::thread> th;
    for (auto& t : ts) th.emplace_back(run_thread, t.get(), cbs);
    for (auto& x : th) x.join();
    std::vector<double> lat;
    uint64_t sent = 0, ok = 0, errors = 0, fail = 0, lost = 0;
    for (auto& t : ts) {
        lat.insert(lat.end(), t->lat_us.begin(), t->lat_us.end());
        sent += t->sent;
        ok += t->ok;
        errors += t->errors;
        fail += t->send_fail;
        lost += t->outstanding;
    }
    const double measured_s = a.seconds;
    const size_t nl = lat.size();
    const double p50 = pct(lat, 50), p99 = pct(lat, 99), p999 = pct(lat, 99.9);
    const double mx = lat.empty() ? NAN : *std::max_element(lat.begin(), lat.end());
    printf("{\"offered_rpc_per_s\": %.1f, \"batch\": %d, \"offered_decisions_per_s\": %.1f, "
           "\"achieved_rpc_per_s\": %.1f, \"achieved_decisions_per_s\": %.1f, \"sent\": %lu, \"completed_ok\": %lu, "
           "\"measured\": %zu, \"errors\": %lu, \"send_failures\": %lu, \"unanswered\": %lu, \"p50_us\": %.1f, "
           "\"p99_us\": %.1f, \"p999_us\": %.1f, \"max_us\": %.1f, \"threads\": %d, \"conns_per_thread\": %d, "
           "\"zipf\": %.2f, \"keys\": %ld, \"limiter\": \"%s\", \"client\": \"rl_grpc_load (C++, nghttp2)\"}\n",
           a.rate, a.batch, a.rate * a.batch, (double)nl / measured_s, (double)nl * a.batch / measured_s,
           (unsigned long)sent, (unsigned long)ok, nl, (unsigned long)errors, (unsigned long)fail,
           (unsigned long)lost, p50, p99, p999, mx, a.threads, a.conns, a.zipf, (long)a.keys, a.limiter.c_str());
    nghttp2_session_callbacks_del(cbs);
    return 0;
}
