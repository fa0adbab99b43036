// ratelimiter.hpp -- host-side mirror of the reference's Go package
// `internal/ratelimiter` over the MI355X engine (include/rl_engine.h).
//
// Same names, argument meaning and error behaviour as the reference:
//   Algorithm / Config / Result        interface.go:8-70
//   Config::Validate / WithDefaults /
//   KeyPrefix / FormatKey              config.go:16-87 (identical messages)
//   RateLimiter::Allow/AllowN/Reset/
//   Close                              interface.go:76-145
//   NewTokenBucket / NewSlidingWindow /
//   NewFixedWindow                     tokenbucket.go:63-81, slidingwindow.go:41-59,
//                                      fixedwindow.go:38-56
//   ErrInvalidN etc.                   errors.go:5-20
// The storage client argument (`*redis.Client`) becomes an `Engine*`; all
// decisions go through one GPU launch sequence (single call or batch).
// Go is not available in this build image; this C++ layer is the executable
// specification of the thin Go/cgo layer shown in INTEGRATION.md.
#pragma once

#include <stdint.h>

#include <atomic>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/rl_engine.h"

namespace ratelimiter {

using Algorithm = std::string;
extern const Algorithm TokenBucket;    // "token_bucket"
extern const Algorithm SlidingWindow;  // "sliding_window"
extern const Algorithm FixedWindow;    // "fixed_window"
extern const char* const DefaultPrefix;  // "ratelimit"

constexpr int64_t Nanosecond = 1, Microsecond = 1000, Millisecond = 1000000, Second = 1000000000,
                  Minute = 60 * Second, Hour = 60 * Minute;

// Go's time.Duration.String()
std::string DurationString(int64_t d);

// Go-style error value: empty = nil.  `is` tags sentinel identity (errors.Is).
struct Error {
    enum Kind { None = 0, InvalidN, InvalidConfig, StorageUnavailable, InvalidKey, Closed, Other };
    Kind is = None;
    std::string msg;
    explicit operator bool() const { return is != None; }
    static Error New(Kind k, std::string m) { return Error{k, std::move(m)}; }
};
extern const Error ErrInvalidConfig, ErrStorageUnavailable, ErrInvalidKey, ErrInvalidN, ErrClosed;

struct Result {
    bool Allowed = false;
    int64_t Limit = 0;
    int64_t Remaining = 0;
    int64_t RetryAfter = 0;  // time.Duration (ns)
    int64_t ResetAt = 0;     // time.Time as Unix ns
};

// time.Time{} (the zero Time) as a ResetAt value
constexpr int64_t ZeroTime = INT64_MIN;

// Result constructors (result.go:5-50)
Result NewAllowedResult(int64_t limit, int64_t remaining, int64_t reset_at);
Result NewDeniedResult(int64_t limit, int64_t retry_after, int64_t reset_at);
Result NewFailOpenResult();
Result NewFailClosedResult();

struct Config {
    Algorithm algorithm;
    int64_t Limit = 0;
    int64_t Window = 0;  // time.Duration (ns)
    std::string Prefix;
    bool FailOpen = false;

    Config WithDefaults() const;
    std::string KeyPrefix() const { return Prefix; }
    std::string FormatKey(const std::string& key) const;
};
// nil-receiver forms (config.go:17-19, :55-57, :72-74)
Error Validate(const Config* c);
std::string KeyPrefix(const Config* c);
std::string FormatKey(const Config* c, const std::string& key);

// context.Context subset: cancellation + deadline (Unix ns, 0 = none)
struct Context {
    std::atomic<bool> cancelled{false};
    int64_t deadline_ns = 0;
    Context() = default;
    Context(const Context& o) : cancelled(o.cancelled.load()), deadline_ns(o.deadline_ns) {}
    static const Context& Background();
};

// Unix-ns clock standing for time.Now(); replaceable for deterministic tests.
using Clock = std::function<int64_t()>;
int64_t WallClockNs();

// One GPU engine plus the key-id interner: the "storage" all limiters share,
// as one Redis.  A key's identity is its formatted name (FormatKey,
// config.go:81-87) and nothing else, so limiters with one Prefix share state
// exactly as they share Redis keys.
class Engine {
public:
    static Error Create(const rl_opts& opts, std::unique_ptr<Engine>* out);
    explicit Engine(rl_engine* e) : e_(e) {}
    ~Engine();
    rl_engine* raw() { return e_; }
    uint64_t Intern(const std::string& formatted_key);
    // the formatted key of an interned id ("" if unknown)
    std::string Name(uint64_t id);
    std::mutex& mu() { return mu_; }
    Clock clock = WallClockNs;
    // test hook: when >= 0, every call passes this Redis clock (ms)
    int64_t server_ms_override = INT64_MIN;

private:
    rl_engine* e_;
    std::mutex mu_;
    std::mutex intern_mu_;
    std::unordered_map<std::string, uint64_t> ids_;
    std::vector<std::string> names_;   // by id
};

struct BatchRequest {
    std::string key;
    int64_t n = 1;
    int64_t now_ns = INT64_MIN;  // INT64_MIN: read the engine clock
};
struct BatchOutcome {
    Error err;
    Result result;
    bool has_result = false;
};

class RateLimiter {
public:
    virtual ~RateLimiter() = default;
    virtual Error Allow(const Context& ctx, const std::string& key, Result* out) = 0;
    virtual Error AllowN(const Context& ctx, const std::string& key, int64_t n, Result* out) = 0;
    virtual Error Reset(const Context& ctx, const std::string& key) = 0;
    // Reset as if called at Unix time t (deterministic replay)
    virtual Error ResetAt(const Context& ctx, const std::string& key, int64_t t) = 0;
    virtual Error Close() = 0;
    // request-coalescing path (new): one engine launch for many requests
    virtual void BatchAllow(const Context& ctx, const std::vector<BatchRequest>& reqs,
                            std::vector<BatchOutcome>* out) = 0;
    virtual const Config& config() const = 0;
};

Error NewTokenBucket(Engine* engine, const Config* config, std::unique_ptr<RateLimiter>* out);
Error NewSlidingWindow(Engine* engine, const Config* config, std::unique_ptr<RateLimiter>* out);
Error NewFixedWindow(Engine* engine, const Config* config, std::unique_ptr<RateLimiter>* out);
// dispatch on config->algorithm
Error New(Engine* engine, const Config* config, std::unique_ptr<RateLimiter>* out);

}  // namespace ratelimiter
