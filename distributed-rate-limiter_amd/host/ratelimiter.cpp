// ratelimiter.cpp -- host mirror of the reference's Go `internal/ratelimiter`
// package over the MI355X engine.  See ratelimiter.hpp for the mapping.
#include "ratelimiter.hpp"
#include "decorators.hpp"

#include <time.h>

#include <cstdio>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>

#include "../../include/rl_limiter.h"
#include "../csrc/rl_semantics.h"

namespace ratelimiter {

const Algorithm TokenBucket = "token_bucket";
const Algorithm SlidingWindow = "sliding_window";
const Algorithm FixedWindow = "fixed_window";
const char* const DefaultPrefix = "ratelimit";

// errors.go:5-20
const Error ErrInvalidConfig{Error::InvalidConfig, "invalid rate limiter configuration"};
const Error ErrStorageUnavailable{Error::StorageUnavailable, "rate limiter storage unavailable"};
const Error ErrInvalidKey{Error::InvalidKey, "invalid key: must not be empty"};
const Error ErrInvalidN{Error::InvalidN, "invalid n: must be greater than 0"};
const Error ErrClosed{Error::Closed, "rate limiter is closed"};

const Context& Context::Background() {
    static Context bg;
    return bg;
}

int64_t WallClockNs() {
    struct timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    return (int64_t)ts.tv_sec * Second + ts.tv_nsec;
}

// ---------------------------------------------------------------------------
// Go time.Duration.String() (time/time.go)
// ---------------------------------------------------------------------------
static int fmt_frac(char* buf, int w, uint64_t* v, int prec) {
    bool print = false;
    for (int i = 0; i < prec; i++) {
        uint64_t digit = *v % 10;
        print = print || digit != 0;
        if (print) buf[--w] = (char)('0' + digit);
        *v /= 10;
    }
    if (print) buf[--w] = '.';
    return w;
}
static int fmt_int(char* buf, int w, uint64_t v) {
    if (v == 0) {
        buf[--w] = '0';
    } else {
        while (v > 0) { buf[--w] = (char)('0' + v % 10); v /= 10; }
    }
    return w;
}

std::string DurationString(int64_t d) {
    char buf[32];
    int w = sizeof buf;
    uint64_t u = (uint64_t)d;
    bool neg = d < 0;
    if (neg) u = -u;
    if (u < (uint64_t)Second) {
        int prec = 0;
        buf[--w] = 's';
        if (u == 0) return "0s";
        if (u < (uint64_t)Microsecond) {
            prec = 0;
            buf[--w] = 'n';
        } else if (u < (uint64_t)Millisecond) {
            prec = 3;
            buf[--w] = '\xb5';  // U+00B5 micro sign, UTF-8 0xC2 0xB5
            buf[--w] = '\xc2';
        } else {
            prec = 6;
            buf[--w] = 'm';
        }
        w = fmt_frac(buf, w, &u, prec);
        w = fmt_int(buf, w, u);
    } else {
        buf[--w] = 's';
        w = fmt_frac(buf, w, &u, 9);
        w = fmt_int(buf, w, u % 60);
        u /= 60;
        if (u > 0) {
            buf[--w] = 'm';
            w = fmt_int(buf, w, u % 60);
            u /= 60;
            if (u > 0) {
                buf[--w] = 'h';
                w = fmt_int(buf, w, u);
            }
        }
    }
    if (neg) buf[--w] = '-';
    return std::string(buf + w, sizeof buf - w);
}

// ---------------------------------------------------------------------------
// Config (config.go)
// ---------------------------------------------------------------------------
Error Validate(const Config* c) {
    if (c == nullptr) return Error::New(Error::Other, "config cannot be nil");
    if (c->algorithm == TokenBucket || c->algorithm == SlidingWindow || c->algorithm == FixedWindow) {
    } else if (c->algorithm.empty()) {
        return Error::New(Error::Other, "algorithm is required");
    } else {
        return Error::New(Error::Other, "unknown algorithm: " + c->algorithm +
                                            " (must be one of: token_bucket, sliding_window, fixed_window)");
    }
    if (c->Limit <= 0) return Error::New(Error::Other, "limit must be greater than 0, got: " + std::to_string(c->Limit));
    if (c->Window <= 0)
        return Error::New(Error::Other, "window must be greater than 0, got: " + DurationString(c->Window));
    if (c->Window < Millisecond)
        return Error::New(Error::Other, "window too small: " + DurationString(c->Window) + " (minimum: 1ms)");
    if (c->Window > 365 * 24 * Hour)
        return Error::New(Error::Other, "window too large: " + DurationString(c->Window) + " (maximum: 365 days)");
    return Error{};
}

Config Config::WithDefaults() const {
    Config r = *this;
    if (r.Prefix.empty()) r.Prefix = DefaultPrefix;
    return r;
}

std::string KeyPrefix(const Config* c) { return c ? c->Prefix : std::string(DefaultPrefix); }

std::string FormatKey(const Config* c, const std::string& key) {
    std::string prefix = KeyPrefix(c);
    if (prefix.empty()) return key;
    return prefix + ":" + key;
}

std::string Config::FormatKey(const std::string& key) const { return ratelimiter::FormatKey(this, key); }

// ---------------------------------------------------------------------------
// Engine
// ---------------------------------------------------------------------------
Error Engine::Create(const rl_opts& opts, std::unique_ptr<Engine>* out) {
    rl_engine* e = nullptr;
    int rc = rl_engine_create(&opts, &e);
    if (rc != RL_OK) return Error::New(Error::StorageUnavailable, "engine create failed: status " + std::to_string(rc));
    out->reset(new Engine(e));
    return Error{};
}

Engine::~Engine() {
    if (e_) rl_engine_destroy(e_);
}

uint64_t Engine::Intern(const std::string& formatted_key) {
    std::lock_guard<std::mutex> g(intern_mu_);
    auto it = ids_.find(formatted_key);
    if (it != ids_.end()) return it->second;
    uint64_t id = names_.size();
    ids_.emplace(formatted_key, id);
    names_.push_back(formatted_key);
    return id;
}

std::string Engine::Name(uint64_t id) {
    std::lock_guard<std::mutex> g(intern_mu_);
    return id < names_.size() ? names_[id] : std::string();
}

// ---------------------------------------------------------------------------
// limiter over the engine: one implementation, three constructors
// ---------------------------------------------------------------------------
namespace {

std::string engine_error(rl_engine* e, int rc) {
    char buf[256] = {0};
    rl_last_error(e, buf, sizeof buf);
    return std::string("engine status ") + std::to_string(rc) + (buf[0] ? std::string(": ") + buf : "");
}

class GpuLimiter final : public RateLimiter {
public:
    GpuLimiter(Engine* eng, Config cfg, uint32_t cfg_id, int32_t alg)
        : eng_(eng), cfg_(std::move(cfg)), cfg_id_(cfg_id),
          host_cfg_(rl::make_cfg(alg, cfg_.Limit, cfg_.Window)) {}

    const Config& config() const override { return cfg_; }

    Error Allow(const Context& ctx, const std::string& key, Result* out) override {
        return AllowN(ctx, key, 1, out);
    }

    Error AllowN(const Context& ctx, const std::string& key, int64_t n, Result* out) override {
        std::vector<BatchRequest> reqs(1);
        reqs[0].key = key;
        reqs[0].n = n;
        std::vector<BatchOutcome> outs;
        BatchAllow(ctx, reqs, &outs);
        if (outs[0].has_result && out) *out = outs[0].result;
        return outs[0].err;
    }

    void BatchAllow(const Context& ctx, const std::vector<BatchRequest>& reqs,
                    std::vector<BatchOutcome>* outs) override {
        size_t m = reqs.size();
        outs->assign(m, BatchOutcome{});
        std::vector<uint64_t> key(m);
        std::vector<int64_t> ts(m), n(m), sms(m);
        std::vector<uint32_t> cfg(m, cfg_id_);
        std::vector<uint8_t> dec(m, rl::DEC_INVALID);
        std::vector<int64_t> rem(m), retry(m), reset(m);
        std::vector<size_t> live;  // requests that reach the engine
        live.reserve(m);
        int64_t clock_now = INT64_MIN;
        for (size_t i = 0; i < m; i++) {
            // AllowN: `if n <= 0 { return nil, ErrInvalidN }` before any I/O
            if (reqs[i].n <= 0) { (*outs)[i].err = ErrInvalidN; continue; }
            int64_t t = reqs[i].now_ns;
            if (t == INT64_MIN) {
                if (clock_now == INT64_MIN) clock_now = eng_->clock();
                t = clock_now;
            }
            size_t k = live.size();
            key[k] = eng_->Intern(cfg_.FormatKey(reqs[i].key));
            ts[k] = t;
            n[k] = reqs[i].n;
            sms[k] = eng_->server_ms_override != INT64_MIN ? eng_->server_ms_override
                                                           : rl::floor_div(t, 1000000LL);
            live.push_back(i);
        }
        if (live.empty()) return;
        std::string cause;
        int rc = RL_OK;
        if (closed_.load()) {
            cause = "engine: client is closed";
            rc = RL_EINVAL;
        } else if (ctx.cancelled.load()) {
            cause = "context canceled";
            rc = RL_EINVAL;
        } else if (ctx.deadline_ns && eng_->clock() >= ctx.deadline_ns) {
            cause = "context deadline exceeded";
            rc = RL_EINVAL;
        } else {
            std::lock_guard<std::mutex> g(eng_->mu());
            rc = rl_decide_batch(eng_->raw(), live.size(), key.data(), ts.data(), n.data(), cfg.data(),
                                 sms.data(), dec.data(), rem.data(), retry.data(), reset.data(), nullptr);
            if (rc != RL_OK) cause = engine_error(eng_->raw(), rc);
        }
        for (size_t k = 0; k < live.size(); k++) {
            BatchOutcome& o = (*outs)[live[k]];
            bool storage_err = rc != RL_OK || dec[k] == rl::DEC_ERROR || dec[k] == rl::DEC_INVALID;
            if (!storage_err) {
                o.has_result = true;
                o.result.Allowed = dec[k] == rl::DEC_ALLOWED;
                o.result.Limit = cfg_.Limit;
                o.result.Remaining = rem[k];
                o.result.RetryAfter = retry[k];
                o.result.ResetAt = reset[k];
                continue;
            }
            std::string why = rc != RL_OK ? cause
                              : dec[k] == rl::DEC_ERROR ? "ERR increment or decrement would overflow"
                                                        : "engine rejected the request";
            if (cfg_.FailOpen) {
                // fail open (tokenbucket.go:101-109, slidingwindow.go:84-92, fixedwindow.go:80-88)
                o.has_result = true;
                o.result.Allowed = true;
                o.result.Limit = cfg_.Limit;
                o.result.Remaining = 0;
                o.result.RetryAfter = 0;
                o.result.ResetAt = fail_open_reset_at(ts[k]);
            } else {
                o.err = Error::New(Error::Other, "failed to check rate limit: " + why);
            }
        }
    }

    Error Reset(const Context& ctx, const std::string& key) override {
        return ResetAt(ctx, key, eng_->clock());
    }

    Error ResetAt(const Context& ctx, const std::string& key, int64_t t) override {
        (void)ctx;
        if (closed_.load())
            return Error::New(Error::Other, "failed to reset rate limit: engine: client is closed");
        uint64_t id = eng_->Intern(cfg_.FormatKey(key));
        std::lock_guard<std::mutex> g(eng_->mu());
        int rc = rl_reset(eng_->raw(), cfg_id_, id, t);
        if (rc != RL_OK)
            return Error::New(Error::Other, "failed to reset rate limit: " + engine_error(eng_->raw(), rc));
        return Error{};
    }

    Error Close() override {
        closed_.store(true);
        return Error{};
    }

private:
    int64_t fail_open_reset_at(int64_t t) const {
        if (host_cfg_.alg == rl::ALG_TOKEN_BUCKET) return rl::tb_reset_at((double)t / 1e9, host_cfg_);
        int64_t ws = rl::window_start(t, host_cfg_);
        return rl::wadd(rl::wmul(ws, rl::NS_PER_S), host_cfg_.window);
    }

    Engine* eng_;
    Config cfg_;
    uint32_t cfg_id_;
    rl::CfgDev host_cfg_;
    std::atomic<bool> closed_{false};
};

int32_t alg_code(const Algorithm& a) {
    if (a == TokenBucket) return rl::ALG_TOKEN_BUCKET;
    if (a == SlidingWindow) return rl::ALG_SLIDING_WINDOW;
    if (a == FixedWindow) return rl::ALG_FIXED_WINDOW;
    return 0;
}

Error construct(Engine* engine, const Config* config, std::unique_ptr<RateLimiter>* out, int32_t alg) {
    if (engine == nullptr) return Error::New(Error::Other, "engine cannot be nil");
    if (config == nullptr) return Error::New(Error::Other, "config cannot be nil");
    Config cfg = config->WithDefaults();
    if (Error err = Validate(&cfg)) return Error::New(Error::Other, "invalid config: " + err.msg);
    if (alg == 0) alg = alg_code(cfg.algorithm);
    uint32_t id = 0;
    int rc;
    {
        std::lock_guard<std::mutex> g(engine->mu());
        rc = rl_config_register(engine->raw(), (uint8_t)alg, cfg.Limit, cfg.Window, &id);
    }
    if (rc != RL_OK) return Error::New(Error::Other, "invalid config: " + engine_error(engine->raw(), rc));
    out->reset(new GpuLimiter(engine, cfg, id, alg));
    return Error{};
}

}  // namespace

// As in the reference, the constructor (not Config.Algorithm) selects the
// algorithm; Config.Algorithm must still pass Validate (tokenbucket.go:71-75).
// result.go:5-50
Result NewAllowedResult(int64_t limit, int64_t remaining, int64_t reset_at) {
    return Result{true, limit, remaining, 0, reset_at};
}
Result NewDeniedResult(int64_t limit, int64_t retry_after, int64_t reset_at) {
    return Result{false, limit, 0, retry_after, reset_at};
}
Result NewFailOpenResult() { return Result{true, 0, 0, 0, ZeroTime}; }
Result NewFailClosedResult() { return Result{false, 0, 0, 0, ZeroTime}; }

Error NewTokenBucket(Engine* e, const Config* c, std::unique_ptr<RateLimiter>* out) {
    return construct(e, c, out, rl::ALG_TOKEN_BUCKET);
}
Error NewSlidingWindow(Engine* e, const Config* c, std::unique_ptr<RateLimiter>* out) {
    return construct(e, c, out, rl::ALG_SLIDING_WINDOW);
}
Error NewFixedWindow(Engine* e, const Config* c, std::unique_ptr<RateLimiter>* out) {
    return construct(e, c, out, rl::ALG_FIXED_WINDOW);
}
Error New(Engine* e, const Config* c, std::unique_ptr<RateLimiter>* out) { return construct(e, c, out, 0); }

}  // namespace ratelimiter

// ===========================================================================
// C-ABI (include/rl_limiter.h)
// ===========================================================================
using namespace ratelimiter;

struct rll_engine {
    std::unique_ptr<Engine> eng;
};
// the LoggingDecorator's records until the caller drains them (pull style:
// no callback into the caller)
class LogQueue {
public:
    explicit LogQueue(size_t cap) : cap_(cap) {}
    void push(std::string line) {
        std::lock_guard<std::mutex> g(mu_);
        if (q_.size() == cap_) {
            q_.pop_front();
            dropped_++;
        }
        q_.push_back(std::move(line));
    }
    int drain(char* buf, size_t len, uint64_t* dropped) {
        std::lock_guard<std::mutex> g(mu_);
        size_t used = 0;
        int n = 0;
        while (!q_.empty() && used + q_.front().size() + 1 <= len) {
            memcpy(buf + used, q_.front().data(), q_.front().size());
            used += q_.front().size();
            q_.pop_front();
            n++;
        }
        if (len) buf[used] = '\0';
        if (dropped) *dropped = dropped_;
        return n;
    }

private:
    std::mutex mu_;
    std::deque<std::string> q_;
    size_t cap_;
    uint64_t dropped_ = 0;
};

struct rll_limiter {
    std::unique_ptr<RateLimiter> lim;
    MetricsDecorator* metrics = nullptr;   // inside lim, when rll_add_metrics wrapped it
    std::shared_ptr<LogQueue> logq;        // rll_add_logging's records
};

static void put_err(char* err, size_t len, const std::string& s) {
    if (err && len) snprintf(err, len, "%s", s.c_str());
}

extern "C" int rll_engine_new(const rl_opts* opts, rll_engine** out, char* err, size_t errlen) {
    if (!opts || !out) return RLL_ERR_ARG;
    auto* h = new rll_engine();
    if (Error e = Engine::Create(*opts, &h->eng)) {
        put_err(err, errlen, e.msg);
        delete h;
        return RLL_ERR_CONFIG;
    }
    *out = h;
    return RLL_OK;
}

extern "C" int rll_engine_free(rll_engine* e) {
    delete e;
    return RLL_OK;
}

extern "C" rl_engine* rll_engine_raw(rll_engine* e) { return e ? e->eng->raw() : nullptr; }

extern "C" int rll_engine_set_server_ms(rll_engine* e, int64_t server_ms) {
    if (!e) return RLL_ERR_ARG;
    e->eng->server_ms_override = server_ms;
    return RLL_OK;
}

extern "C" int rll_keys(rll_engine* e, int64_t server_ms, char* buf, size_t len) {
    if (!e || (len && !buf)) return -RLL_ERR_ARG;
    std::vector<rl_key_rec> recs(64);
    uint64_t n = 0;
    for (;;) {
        std::lock_guard<std::mutex> g(e->eng->mu());
        if (rl_table_keys(e->eng->raw(), server_ms, recs.data(), recs.size(), &n) != RL_OK) return -RLL_ERR_FAILED;
        if (n <= recs.size()) break;
        recs.resize(n);
    }
    std::vector<std::string> names;
    for (uint64_t i = 0; i < n; i++) {
        std::string b = e->eng->Name(recs[i].key_id);
        // a window key: fmt.Sprintf("%s:%d", FormatKey(key), ws) (fixedwindow.go:139-141)
        if (recs[i].kind == RL_KIND_WINDOW) b += ":" + std::to_string(recs[i].window_start);
        names.push_back(std::move(b));
    }
    std::sort(names.begin(), names.end());
    std::string out;
    for (auto& x : names) out += x + "\n";
    if (len) snprintf(buf, len, "%s", out.c_str());
    return (int)out.size();
}

extern "C" int rll_config_validate(const char* algorithm, int64_t limit, int64_t window_ns, char* err,
                                   size_t errlen) {
    if (!algorithm) {
        put_err(err, errlen, Validate(nullptr).msg);
        return RLL_ERR_CONFIG;
    }
    Config c;
    c.algorithm = algorithm;
    c.Limit = limit;
    c.Window = window_ns;
    if (Error e = Validate(&c)) {
        put_err(err, errlen, e.msg);
        return RLL_ERR_CONFIG;
    }
    return RLL_OK;
}

extern "C" int rll_format_key(const char* prefix, const char* key, char* out, size_t len) {
    Config c;
    if (prefix) c.Prefix = prefix;
    std::string r = FormatKey(prefix ? &c : nullptr, key ? key : "");
    put_err(out, len, r);
    return (int)r.size();
}

extern "C" int rll_duration_string(int64_t d, char* out, size_t len) {
    std::string r = DurationString(d);
    put_err(out, len, r);
    return (int)r.size();
}

extern "C" int rll_new(rll_engine* e, const char* algorithm, int64_t limit, int64_t window_ns,
                       const char* prefix, int fail_open, int config_nil, rll_limiter** out, char* err,
                       size_t errlen) {
    if (!out) return RLL_ERR_ARG;
    *out = nullptr;
    Config c;
    c.algorithm = algorithm ? algorithm : "";
    c.Limit = limit;
    c.Window = window_ns;
    c.Prefix = prefix ? prefix : "";
    c.FailOpen = fail_open != 0;
    auto* h = new rll_limiter();
    Error er = New(e ? e->eng.get() : nullptr, config_nil ? nullptr : &c, &h->lim);
    if (er) {
        put_err(err, errlen, er.msg);
        delete h;
        return RLL_ERR_CONFIG;
    }
    *out = h;
    return RLL_OK;
}

static void to_c(const Result& r, rll_result* o) {
    o->allowed = r.Allowed ? 1 : 0;
    o->limit = r.Limit;
    o->remaining = r.Remaining;
    o->retry_after_ns = r.RetryAfter;
    o->reset_at_ns = r.ResetAt;
}

extern "C" int rll_add_metrics(rll_limiter* l) {
    if (!l || !l->lim || l->metrics) return RLL_ERR_ARG;
    auto* m = new MetricsDecorator(std::move(l->lim));
    l->lim.reset(m);
    l->metrics = m;
    return RLL_OK;
}

extern "C" int rll_metrics_expose(rll_limiter* l, char* buf, size_t len) {
    if (!l || !l->metrics) return -RLL_ERR_ARG;
    const std::string s = l->metrics->Expose();
    if (buf && len) snprintf(buf, len, "%s", s.c_str());
    return (int)s.size();
}

extern "C" int rll_add_logging(rll_limiter* l, size_t capacity) {
    if (!l || !l->lim || capacity == 0 || l->logq) return RLL_ERR_ARG;
    auto q = std::make_shared<LogQueue>(capacity);
    l->logq = q;
    l->lim.reset(new LoggingDecorator(
        std::move(l->lim),
        [q](LogLevel lv, const std::string& msg, const std::vector<std::pair<std::string, std::string>>& f) {
            std::string kv;
            for (const auto& p : f) kv += (kv.empty() ? "" : " ") + p.first + "=" + p.second;
            q->push(std::to_string((int)lv) + "\t" + msg + "\t" + kv + "\n");
        }));
    return RLL_OK;
}

extern "C" int rll_log_drain(rll_limiter* l, char* buf, size_t len, uint64_t* dropped) {
    if (!l || !l->logq || (len && !buf)) return -RLL_ERR_ARG;
    return l->logq->drain(buf, len, dropped);
}

extern "C" int rll_new_allowed_result(int64_t limit, int64_t remaining, int64_t reset_at_ns, rll_result* out) {
    if (!out) return RLL_ERR_ARG;
    to_c(NewAllowedResult(limit, remaining, reset_at_ns), out);
    return RLL_OK;
}

extern "C" int rll_new_denied_result(int64_t limit, int64_t retry_after_ns, int64_t reset_at_ns, rll_result* out) {
    if (!out) return RLL_ERR_ARG;
    to_c(NewDeniedResult(limit, retry_after_ns, reset_at_ns), out);
    return RLL_OK;
}

extern "C" int rll_new_fail_open_result(rll_result* out) {
    if (!out) return RLL_ERR_ARG;
    to_c(NewFailOpenResult(), out);
    return RLL_OK;
}

extern "C" int rll_new_fail_closed_result(rll_result* out) {
    if (!out) return RLL_ERR_ARG;
    to_c(NewFailClosedResult(), out);
    return RLL_OK;
}

static int code_of(const Error& e) {
    if (!e) return RLL_OK;
    if (e.is == Error::InvalidN) return RLL_ERR_INVALID_N;
    return RLL_ERR_FAILED;
}

extern "C" int rll_allow_n(rll_limiter* l, const char* key, size_t keylen, int64_t n, int64_t now_ns,
                           int ctx_cancelled, rll_result* out, char* err, size_t errlen) {
    if (!l || (!key && keylen)) return RLL_ERR_ARG;
    Context ctx;
    ctx.cancelled.store(ctx_cancelled != 0);
    std::vector<BatchRequest> reqs(1);
    reqs[0].key.assign(key ? key : "", keylen);
    reqs[0].n = n;
    reqs[0].now_ns = now_ns;
    std::vector<BatchOutcome> outs;
    l->lim->BatchAllow(ctx, reqs, &outs);
    if (outs[0].has_result && out) to_c(outs[0].result, out);
    if (outs[0].err) put_err(err, errlen, outs[0].err.msg);
    return code_of(outs[0].err);
}

extern "C" int rll_allow_batch(rll_limiter* l, size_t m, const char* const* keys, const size_t* keylens,
                               const int64_t* n, const int64_t* now_ns, rll_result* out, int32_t* codes) {
    if (!l || (m && (!keys || !keylens || !n || !out || !codes))) return RLL_ERR_ARG;
    std::vector<BatchRequest> reqs(m);
    for (size_t i = 0; i < m; i++) {
        reqs[i].key.assign(keys[i], keylens[i]);
        reqs[i].n = n[i];
        reqs[i].now_ns = now_ns ? now_ns[i] : INT64_MIN;
    }
    std::vector<BatchOutcome> outs;
    l->lim->BatchAllow(Context::Background(), reqs, &outs);
    for (size_t i = 0; i < m; i++) {
        if (outs[i].has_result) to_c(outs[i].result, &out[i]);
        else memset(&out[i], 0, sizeof out[i]);
        codes[i] = code_of(outs[i].err);
    }
    return RLL_OK;
}

extern "C" int rll_reset(rll_limiter* l, const char* key, size_t keylen, int64_t now_ns, char* err,
                         size_t errlen) {
    if (!l || (!key && keylen)) return RLL_ERR_ARG;
    std::string k(key ? key : "", keylen);
    Error e = now_ns == RLL_NOW_WALL ? l->lim->Reset(Context::Background(), k)
                                     : l->lim->ResetAt(Context::Background(), k, now_ns);
    if (e) {
        put_err(err, errlen, e.msg);
        return RLL_ERR_RESET;
    }
    return RLL_OK;
}

extern "C" int rll_close(rll_limiter* l) {
    if (!l) return RLL_ERR_ARG;
    l->lim->Close();
    return RLL_OK;
}

extern "C" int rll_free(rll_limiter* l) {
    delete l;
    return RLL_OK;
}
