// decorators.hpp -- observability decorators over any RateLimiter, as the
// reference designs them (docs/ADR/003-decorator-pattern-for-observability.md:
// 26-125): the core limiter stays free of metrics and
// logging, and each concern wraps it with the same interface.
//
//   MetricsDecorator   requests counted by (algorithm, allowed, error type) and
//                      a decision-latency histogram, exposed in the Prometheus
//                      text format (ADR-003:37-58)
//   LoggingDecorator   errors at Error level, denials at Debug level, through a
//                      caller-supplied sink (ADR-003:62-83)
#pragma once

#include <stdint.h>

#include <array>
#include <atomic>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "ratelimiter.hpp"

namespace ratelimiter {

// getErrorType of ADR-003:49: a label value per error kind
const char* ErrorType(const Error& e);

class MetricsDecorator : public RateLimiter {
public:
    explicit MetricsDecorator(std::unique_ptr<RateLimiter> inner, Clock clock = WallClockNs);
    Error Allow(const Context& ctx, const std::string& key, Result* out) override;
    Error AllowN(const Context& ctx, const std::string& key, int64_t n, Result* out) override;
    Error Reset(const Context& ctx, const std::string& key) override;
    Error ResetAt(const Context& ctx, const std::string& key, int64_t t) override;
    Error Close() override { return inner_->Close(); }
    void BatchAllow(const Context& ctx, const std::vector<BatchRequest>& reqs,
                    std::vector<BatchOutcome>* out) override;
    const Config& config() const override { return inner_->config(); }

    // rate_limiter_requests_total{algorithm,allowed,error} and
    // rate_limiter_decision_seconds (histogram), Prometheus text format
    std::string Expose() const;
    uint64_t Count(bool allowed, const std::string& error) const;

    // histogram bucket upper bounds, seconds (10 us .. 1 s)
    static const std::array<double, 12> kBuckets;

private:
    void record(const Error& e, const Result* r, int64_t n_decisions, int64_t elapsed_ns);
    std::unique_ptr<RateLimiter> inner_;
    Clock clock_;
    mutable std::mutex mu_;
    std::map<std::pair<bool, std::string>, uint64_t> requests_;
    std::array<uint64_t, 13> hist_{};   // kBuckets + +Inf
    double sum_s_ = 0.0;
    uint64_t observations_ = 0;
};

enum class LogLevel { Debug = 0, Info = 1, Warn = 2, Error = 3 };
// one structured record: message plus key/value fields
using LogSink = std::function<void(LogLevel, const std::string& msg,
                                   const std::vector<std::pair<std::string, std::string>>& fields)>;

class LoggingDecorator : public RateLimiter {
public:
    LoggingDecorator(std::unique_ptr<RateLimiter> inner, LogSink sink);
    Error Allow(const Context& ctx, const std::string& key, Result* out) override;
    Error AllowN(const Context& ctx, const std::string& key, int64_t n, Result* out) override;
    Error Reset(const Context& ctx, const std::string& key) override;
    Error ResetAt(const Context& ctx, const std::string& key, int64_t t) override;
    Error Close() override { return inner_->Close(); }
    void BatchAllow(const Context& ctx, const std::vector<BatchRequest>& reqs,
                    std::vector<BatchOutcome>* out) override;
    const Config& config() const override { return inner_->config(); }

private:
    void log_outcome(const std::string& key, const Error& e, const Result* r);
    std::unique_ptr<RateLimiter> inner_;
    LogSink sink_;
};

}  // namespace ratelimiter
