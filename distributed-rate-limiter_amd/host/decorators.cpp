// decorators.cpp -- see decorators.hpp (ADR-003 decorator pattern).
#include "decorators.hpp"

#include <stdio.h>

namespace ratelimiter {

const char* ErrorType(const Error& e) {
    switch (e.is) {
        case Error::None: return "none";
        case Error::InvalidN: return "invalid_n";
        case Error::InvalidConfig: return "invalid_config";
        case Error::StorageUnavailable: return "storage_unavailable";
        case Error::InvalidKey: return "invalid_key";
        case Error::Closed: return "closed";
        default: return "other";
    }
}

const std::array<double, 12> MetricsDecorator::kBuckets = {1e-5, 2.5e-5, 5e-5, 1e-4, 2.5e-4, 5e-4,
                                                          1e-3, 2.5e-3, 5e-3, 1e-2, 1e-1, 1.0};

MetricsDecorator::MetricsDecorator(std::unique_ptr<RateLimiter> inner, Clock clock)
    : inner_(std::move(inner)), clock_(std::move(clock)) {}

void MetricsDecorator::record(const Error& e, const Result* r, int64_t n_decisions, int64_t elapsed_ns) {
    const double s = (double)elapsed_ns / 1e9;
    size_t b = 0;
    while (b < kBuckets.size() && s > kBuckets[b]) b++;
    std::lock_guard<std::mutex> g(mu_);
    requests_[{!e && r && r->Allowed, ErrorType(e)}] += 1;
    hist_[b] += (uint64_t)n_decisions;
    sum_s_ += s * (double)n_decisions;
    observations_ += (uint64_t)n_decisions;
}

Error MetricsDecorator::Allow(const Context& ctx, const std::string& key, Result* out) {
    return AllowN(ctx, key, 1, out);
}

Error MetricsDecorator::AllowN(const Context& ctx, const std::string& key, int64_t n, Result* out) {
    const int64_t t0 = clock_();
    Result r;
    Error e = inner_->AllowN(ctx, key, n, &r);
    record(e, &r, 1, clock_() - t0);
    if (!e && out) *out = r;
    return e;
}

Error MetricsDecorator::Reset(const Context& ctx, const std::string& key) { return inner_->Reset(ctx, key); }
Error MetricsDecorator::ResetAt(const Context& ctx, const std::string& key, int64_t t) {
    return inner_->ResetAt(ctx, key, t);
}

void MetricsDecorator::BatchAllow(const Context& ctx, const std::vector<BatchRequest>& reqs,
                                  std::vector<BatchOutcome>* out) {
    const int64_t t0 = clock_();
    inner_->BatchAllow(ctx, reqs, out);
    const int64_t dt = clock_() - t0;
    // every request of the batch waited for the whole batch
    for (const auto& o : *out) record(o.err, o.has_result ? &o.result : nullptr, 1, dt);
}

uint64_t MetricsDecorator::Count(bool allowed, const std::string& error) const {
    std::lock_guard<std::mutex> g(mu_);
    auto it = requests_.find({allowed, error});
    return it == requests_.end() ? 0 : it->second;
}

std::string MetricsDecorator::Expose() const {
    std::lock_guard<std::mutex> g(mu_);
    const std::string alg = inner_->config().algorithm;
    std::string s = "# HELP rate_limiter_requests_total Rate limit decisions by outcome.\n"
                    "# TYPE rate_limiter_requests_total counter\n";
    char line[256];
    for (const auto& kv : requests_) {
        snprintf(line, sizeof line, "rate_limiter_requests_total{algorithm=\"%s\",allowed=\"%s\",error=\"%s\"} %llu\n",
                 alg.c_str(), kv.first.first ? "true" : "false", kv.first.second.c_str(),
                 (unsigned long long)kv.second);
        s += line;
    }
    s += "# HELP rate_limiter_decision_seconds Decision latency.\n"
         "# TYPE rate_limiter_decision_seconds histogram\n";
    uint64_t acc = 0;
    for (size_t b = 0; b <= kBuckets.size(); b++) {
        acc += hist_[b];
        if (b < kBuckets.size())
            snprintf(line, sizeof line, "rate_limiter_decision_seconds_bucket{algorithm=\"%s\",le=\"%g\"} %llu\n",
                     alg.c_str(), kBuckets[b], (unsigned long long)acc);
        else
            snprintf(line, sizeof line, "rate_limiter_decision_seconds_bucket{algorithm=\"%s\",le=\"+Inf\"} %llu\n",
                     alg.c_str(), (unsigned long long)acc);
        s += line;
    }
    snprintf(line, sizeof line, "rate_limiter_decision_seconds_sum{algorithm=\"%s\"} %.9g\n", alg.c_str(), sum_s_);
    s += line;
    snprintf(line, sizeof line, "rate_limiter_decision_seconds_count{algorithm=\"%s\"} %llu\n", alg.c_str(),
             (unsigned long long)observations_);
    s += line;
    return s;
}

LoggingDecorator::LoggingDecorator(std::unique_ptr<RateLimiter> inner, LogSink sink)
    : inner_(std::move(inner)), sink_(std::move(sink)) {}

void LoggingDecorator::log_outcome(const std::string& key, const Error& e, const Result* r) {
    if (e) {
        sink_(LogLevel::Error, "rate limiter error", {{"key", key}, {"error", e.msg}});
    } else if (r && !r->Allowed) {
        sink_(LogLevel::Debug, "request denied", {{"key", key}, {"limit", std::to_string(r->Limit)}});
    }
}

Error LoggingDecorator::Allow(const Context& ctx, const std::string& key, Result* out) {
    return AllowN(ctx, key, 1, out);
}

Error LoggingDecorator::AllowN(const Context& ctx, const std::string& key, int64_t n, Result* out) {
    Result r;
    Error e = inner_->AllowN(ctx, key, n, &r);
    log_outcome(key, e, e ? nullptr : &r);
    if (!e && out) *out = r;
    return e;
}

Error LoggingDecorator::Reset(const Context& ctx, const std::string& key) {
    Error e = inner_->Reset(ctx, key);
    if (e) sink_(LogLevel::Error, "rate limiter reset error", {{"key", key}, {"error", e.msg}});
    return e;
}

Error LoggingDecorator::ResetAt(const Context& ctx, const std::string& key, int64_t t) {
    Error e = inner_->ResetAt(ctx, key, t);
    if (e) sink_(LogLevel::Error, "rate limiter reset error", {{"key", key}, {"error", e.msg}});
    return e;
}

void LoggingDecorator::BatchAllow(const Context& ctx, const std::vector<BatchRequest>& reqs,
                                  std::vector<BatchOutcome>* out) {
    inner_->BatchAllow(ctx, reqs, out);
    for (size_t i = 0; i < out->size(); i++)
        log_outcome(reqs[i].key, (*out)[i].err, (*out)[i].has_result ? &(*out)[i].result : nullptr);
}

}  // namespace ratelimiter
