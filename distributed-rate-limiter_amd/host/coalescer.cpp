// coalescer.cpp -- see coalescer.hpp / include/rl_coalescer.h.
#include "coalescer.hpp"

#include <hip/hip_runtime.h>
#include <string.h>

#include <stdlib.h>

#include <algorithm>
#include <chrono>

namespace rlc {

int64_t steady_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

// per request: key 8 + ts 8 + n 8 + rem 8 + retry 8 + reset 8 + cfg 4 + dec 1
Sub::Sub(size_t m_) : mem(new uint8_t[(m_ ? m_ : 1) * 53 + 8]), cap(m_ ? m_ : 1) { carve(m_); }

void Sub::carve(size_t m_) {
    first = 0;
    m = m_;
    taken = 0;
    left = m_;
    status = RL_OK;
    reset_op = done = waiting = false;
    done_ns = submit_ns = 0;
    // layout by capacity, so a reused buffer keeps its arrays in place
    const size_t c = cap;
    uint8_t* p = mem.get();
    key = reinterpret_cast<uint64_t*>(p);
    ts = reinterpret_cast<int64_t*>(p + 8 * c);
    n = reinterpret_cast<int64_t*>(p + 16 * c);
    rem = reinterpret_cast<int64_t*>(p + 24 * c);
    retry = reinterpret_cast<int64_t*>(p + 32 * c);
    reset = reinterpret_cast<int64_t*>(p + 40 * c);
    cfg = reinterpret_cast<uint32_t*>(p + 48 * c);
    dec = p + 52 * c;
}

// Completion waits: the runtime's (default), or polling the event
// (RL_COALESCER_POLL=1, one busy core per waiting thread).  The A/B in
// DESIGN.md (configs[4] tail) found the same rare stalls either way.
static bool poll_waits() {
    static const bool p = getenv("RL_COALESCER_POLL") != nullptr;
    return p;
}
static hipError_t await_event(hipEvent_t ev) {
    if (!poll_waits()) return hipEventSynchronize(ev);
    for (;;) {
        const hipError_t r = hipEventQuery(ev);
        if (r != hipErrorNotReady) return r;
        for (int i = 0; i < 32; i++) __builtin_ia32_pause();
    }
}

// ---------------------------------------------------------------------------
// GPU backend: pinned staging per slot, one H2D copy stream, results come back
// on an output stream that the engine orders behind each batch's finish.
// Inputs are complete when rl_decide_batch_device is called (the H2D copy is
// waited for on the submitter thread), so an engine created with
// RL_OPT_PIPELINE overlaps batch b+1's grouping with batch b's replay.
// ---------------------------------------------------------------------------
class GpuBackend : public Backend {
public:
    explicit GpuBackend(rl_engine* e) : e_(e) { (void)hipGetDevice(&dev_id_); }
    ~GpuBackend() override {
        for (auto& d : dev_) {
            (void)hipFree(d.key);
            if (d.ev) (void)hipEventDestroy(d.ev);
            if (d.ev_in) (void)hipEventDestroy(d.ev_in);
        }
        for (void* h : host_) (void)hipHostFree(h);
        if (cs_) (void)hipStreamDestroy(cs_);
        if (os_) (void)hipStreamDestroy(os_);
    }
    int init(int nslots, size_t M, std::vector<Slot>* slots) override {
        (void)hipSetDevice(dev_id_);
        if (hipStreamCreateWithFlags(&cs_, hipStreamNonBlocking) != hipSuccess) return RL_EDEVICE;
        if (hipStreamCreateWithFlags(&os_, hipStreamNonBlocking) != hipSuccess) return RL_EDEVICE;
        slots->resize(nslots);
        dev_.resize(nslots);
        for (int i = 0; i < nslots; i++) {
            // inputs first (one H2D block), then outputs
            void* h = nullptr;
            if (hipHostMalloc(&h, M * 61 + 64, hipHostMallocDefault) != hipSuccess) return RL_ENOMEM;
            host_.push_back(h);
            carve(static_cast<uint8_t*>(h), M, (*slots)[i]);
            Dev& d = dev_[i];
            uint8_t* dp = nullptr;
            if (hipMalloc(&dp, M * 61 + 64) != hipSuccess) return RL_ENOMEM;
            d.key = dp;
            if (hipEventCreateWithFlags(&d.ev, hipEventDisableTiming) != hipSuccess) return RL_EDEVICE;
            if (hipEventCreateWithFlags(&d.ev_in, hipEventDisableTiming) != hipSuccess) return RL_EDEVICE;
        }
        M_ = M;
        return RL_OK;
    }
    int launch(int i, Slot& s) override {
        (void)hipSetDevice(dev_id_);   // the submitter thread
        Dev& d = dev_[i];
        Slot dv;
        carve(d.key, M_, dv);
        const size_t m = s.m;
        bool ok = hipMemcpyAsync(dv.key, s.key, 8 * m, hipMemcpyHostToDevice, cs_) == hipSuccess;
        ok &= hipMemcpyAsync(dv.ts, s.ts, 8 * m, hipMemcpyHostToDevice, cs_) == hipSuccess;
        ok &= hipMemcpyAsync(dv.n, s.n, 8 * m, hipMemcpyHostToDevice, cs_) == hipSuccess;
        ok &= hipMemcpyAsync(dv.cfg, s.cfg, 4 * m, hipMemcpyHostToDevice, cs_) == hipSuccess;
        ok &= hipEventRecord(d.ev_in, cs_) == hipSuccess;
        ok &= await_event(d.ev_in) == hipSuccess;
        if (!ok) return RL_EDEVICE;
        s.t_h2d = steady_ns();
        int rc = rl_decide_batch_device(e_, m, dv.key, dv.ts, dv.n, dv.cfg, nullptr, dv.dec, dv.rem, dv.retry,
                                        dv.reset, nullptr, os_);
        if (rc != RL_OK) return rc;
        ok = hipMemcpyAsync(s.dec, dv.dec, m, hipMemcpyDeviceToHost, os_) == hipSuccess;
        ok &= hipMemcpyAsync(s.rem, dv.rem, 8 * m, hipMemcpyDeviceToHost, os_) == hipSuccess;
        ok &= hipMemcpyAsync(s.retry, dv.retry, 8 * m, hipMemcpyDeviceToHost, os_) == hipSuccess;
        ok &= hipMemcpyAsync(s.reset, dv.reset, 8 * m, hipMemcpyDeviceToHost, os_) == hipSuccess;
        ok &= hipEventRecord(d.ev, os_) == hipSuccess;
        return ok ? RL_OK : RL_EDEVICE;
    }
    int wait(int i, Slot&) override {
        (void)hipSetDevice(dev_id_);   // the completer thread
        return await_event(dev_[i].ev) == hipSuccess ? RL_OK : RL_EDEVICE;
    }
    int reset(uint32_t cfg, uint64_t key, int64_t ts) override {
        (void)hipSetDevice(dev_id_);   // the submitter thread
        return rl_reset(e_, cfg, key, ts);
    }

private:
    struct Dev {
        uint8_t* key = nullptr;   // base of the slot's device block
        hipEvent_t ev = nullptr;       // results back on the host
        hipEvent_t ev_in = nullptr;    // inputs on the device
    };
    // SoA layout of one slot block: key ts n | cfg | rem retry reset | dec
    static void carve(uint8_t* p, size_t M, Slot& s) {
        s.key = reinterpret_cast<uint64_t*>(p);
        s.ts = reinterpret_cast<int64_t*>(p + 8 * M);
        s.n = reinterpret_cast<int64_t*>(p + 16 * M);
        s.cfg = reinterpret_cast<uint32_t*>(p + 24 * M);
        uint8_t* q = p + ((28 * M + 63) & ~size_t(63));
        s.rem = reinterpret_cast<int64_t*>(q);
        s.retry = reinterpret_cast<int64_t*>(q + 8 * M);
        s.reset = reinterpret_cast<int64_t*>(q + 16 * M);
        s.dec = q + 24 * M;
    }
    rl_engine* e_;
    int dev_id_ = 0;             // the engine's device: current when the coalescer is created
    hipStream_t cs_ = nullptr, os_ = nullptr;
    std::vector<void*> host_;
    std::vector<Dev> dev_;
    size_t M_ = 0;
};

// synchronous host function (the CPU tests plug the oracle in here)
class FnBackend : public Backend {
public:
    FnBackend(rl_batch_fn fn, rl_reset_fn rfn, void* user) : fn_(fn), rfn_(rfn), user_(user) {}
    int init(int nslots, size_t M, std::vector<Slot>* slots) override {
        slots->resize(nslots);
        mem_.resize(nslots);
        for (int i = 0; i < nslots; i++) {
            mem_[i].reset(new uint8_t[M * 61 + 64]);
            uint8_t* p = mem_[i].get();
            Slot& s = (*slots)[i];
            s.key = reinterpret_cast<uint64_t*>(p);
            s.ts = reinterpret_cast<int64_t*>(p + 8 * M);
            s.n = reinterpret_cast<int64_t*>(p + 16 * M);
            s.rem = reinterpret_cast<int64_t*>(p + 24 * M);
            s.retry = reinterpret_cast<int64_t*>(p + 32 * M);
            s.reset = reinterpret_cast<int64_t*>(p + 40 * M);
            s.cfg = reinterpret_cast<uint32_t*>(p + 48 * M);
            s.dec = p + 52 * M;
        }
        return RL_OK;
    }
    int launch(int, Slot& s) override {
        s.t_h2d = steady_ns();
        return fn_(user_, s.m, s.key, s.ts, s.n, s.cfg, s.dec, s.rem, s.retry, s.reset);
    }
    int wait(int, Slot&) override { return RL_OK; }
    int reset(uint32_t cfg, uint64_t key, int64_t ts) override {
        return rfn_ ? rfn_(user_, cfg, key, ts) : RL_EINVAL;
    }

private:
    rl_batch_fn fn_;
    rl_reset_fn rfn_;
    void* user_;
    std::vector<std::unique_ptr<uint8_t[]>> mem_;
};

std::unique_ptr<Backend> make_gpu_backend(rl_engine* e) { return std::unique_ptr<Backend>(new GpuBackend(e)); }
std::unique_ptr<Backend> make_fn_backend(rl_batch_fn fn, rl_reset_fn rfn, void* user) {
    return std::unique_ptr<Backend>(new FnBackend(fn, rfn, user));
}

// ---------------------------------------------------------------------------

Coalescer::Coalescer(std::unique_ptr<Backend> be, const rl_coalescer_opts& o) : be_(std::move(be)), o_(o) {
    if (o_.max_batch == 0) o_.max_batch = 65536;
    if (o_.max_in_flight == 0) o_.max_in_flight = 3;
    if (o_.max_in_flight > 3) o_.max_in_flight = 3;
    if (o_.queue_cap == 0) o_.queue_cap = 1ull << 24;
    if (o_.linger_ns < 0) o_.linger_ns = 0;
    if (const char* v = getenv("RL_COALESCER_TRACE")) trace_cap_ = (size_t)strtoull(v, nullptr, 10);
}

int Coalescer::start() {
    int rc = be_->init((int)o_.max_in_flight, o_.max_batch, &slots_);
    if (rc != RL_OK) return rc;
    t_sub_ = std::thread([this] { submitter(); });
    t_done_ = std::thread([this] { completer(); });
    return RL_OK;
}

Coalescer::~Coalescer() {
    Shutdown();
    for (auto& kv : subs_) delete kv.second;
    for (Sub* s : pool_) delete s;
}

void Coalescer::Shutdown() {
    {
        std::lock_guard<std::mutex> g(mu_);
        if (stop_) return;
        stop_ = true;
    }
    cv_sub_.notify_all();
    cv_done_.notify_all();
    if (t_sub_.joinable()) t_sub_.join();
    if (t_done_.joinable()) t_done_.join();
    // anything never launched (backend failure) is released as closed
    std::lock_guard<std::mutex> g(mu_);
    for (auto& kv : subs_) {
        Sub* s = kv.second;
        if (!s->done) {
            s->done = true;
            s->status = RL_ECLOSED;
            s->cv.notify_all();
        }
    }
}

int Coalescer::Submit(size_t m, const uint64_t* key, const int64_t* ts, const int64_t* n, const uint32_t* cfg,
                      uint64_t* ticket, bool reset_op) {
    if (!ticket || (m && (!key || !ts || !n || !cfg)) || (reset_op && m != 1)) return RL_EINVAL;
    Sub* s = get_sub(m);
    s->reset_op = reset_op;
    if (trace_cap_) s->submit_ns = steady_ns();
    memcpy(s->key, key, 8 * m);
    memcpy(s->ts, ts, 8 * m);
    memcpy(s->n, n, 8 * m);
    memcpy(s->cfg, cfg, 4 * m);
    {
        std::lock_guard<std::mutex> g(mu_);
        if (stop_ || pending_ + m > o_.queue_cap) {
            const int rc = stop_ ? RL_ECLOSED : RL_EAGAIN;
            put_sub(s);
            return rc;
        }
        s->first = next_seq_;
        // an empty submission is done at once; its ticket must still be unique
        next_seq_ += m ? m : 1;
        subs_[s->first] = s;
        st_.submitted += m;
        if (m) {
            queue_.push_back(s);
            pending_ += m;
        } else {
            s->done = true;
            s->done_ns = steady_ns();
        }
        *ticket = s->first;
        // wake the submitter only when it sleeps: at millions of submissions
        // per second an unconditional notify is a futex call per submission
        if (!m || !sub_idle_) return RL_OK;
    }
    cv_sub_.notify_one();
    return RL_OK;
}

int Coalescer::Wait(uint64_t ticket, int64_t timeout_ns, uint8_t* dec, int64_t* rem, int64_t* retry,
                    int64_t* reset, int64_t* done_ns) {
    std::unique_lock<std::mutex> lk(mu_);
    auto it = subs_.find(ticket);
    if (it == subs_.end()) return RL_EINVAL;
    Sub* s = it->second;
    if (!s->done) {
        s->waiting = true;
        if (timeout_ns < 0) {
            s->cv.wait(lk, [&] { return s->done; });
        } else if (!s->cv.wait_for(lk, std::chrono::nanoseconds(timeout_ns), [&] { return s->done; })) {
            s->waiting = false;
            return RL_ETIMEOUT;
        }
    }
    subs_.erase(it);
    lk.unlock();
    const size_t m = s->m;
    if (dec) memcpy(dec, s->dec, m);
    if (rem) memcpy(rem, s->rem, 8 * m);
    if (retry) memcpy(retry, s->retry, 8 * m);
    if (reset) memcpy(reset, s->reset, 8 * m);
    if (done_ns) *done_ns = s->done_ns;
    int st = s->status;
    put_sub(s);
    return st;
}

Sub* Coalescer::get_sub(size_t m) {
    {
        std::lock_guard<std::mutex> g(pool_mu_);
        for (size_t i = pool_.size(); i-- > 0;) {
            Sub* s = pool_[i];
            if (s->cap >= m && s->cap <= 4 * m + 4096) {   // fits, and not far too big
                pool_[i] = pool_.back();
                pool_.pop_back();
                s->carve(m);
                return s;
            }
        }
    }
    return new Sub(m);
}

void Coalescer::put_sub(Sub* s) {
    {
        std::lock_guard<std::mutex> g(pool_mu_);
        if (pool_.size() < 256 && s->cap <= (1u << 20)) {
            pool_.push_back(s);
            return;
        }
    }
    delete s;
}

std::vector<BatchTrace> Coalescer::Trace() {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<BatchTrace> out;
    if (trace_.size() < trace_cap_) return trace_;
    const size_t h = done_batches_ % trace_cap_;
    out.insert(out.end(), trace_.begin() + h, trace_.end());
    out.insert(out.end(), trace_.begin(), trace_.begin() + h);
    return out;
}

rl_coalescer_stats Coalescer::Stats() {
    std::lock_guard<std::mutex> g(mu_);
    rl_coalescer_stats r = st_;
    r.pending = pending_;
    return r;
}

void Coalescer::submitter() {
    for (;;) {
        std::unique_lock<std::mutex> lk(mu_);
        sub_idle_ = true;
        cv_sub_.wait(lk, [&] { return (stop_ && pending_ == 0) || (pending_ > 0 && inflight_ < (int)o_.max_in_flight); });
        sub_idle_ = false;
        if (pending_ == 0) break;   // stop_ with nothing left
        if (o_.linger_ns > 0 && inflight_ == 0 && pending_ < o_.max_batch && !stop_ && !queue_.front()->reset_op) {
            const auto until = std::chrono::steady_clock::now() + std::chrono::nanoseconds(o_.linger_ns);
            sub_idle_ = true;
            cv_sub_.wait_until(lk, until, [&] { return stop_ || pending_ >= o_.max_batch; });
            sub_idle_ = false;
        }
        if (queue_.front()->reset_op) {
            // every request before it is launched; the backend's reset waits
            // for them on the device, then applies the DEL
            Sub* r = queue_.front();
            queue_.pop_front();
            pending_ -= 1;
            r->taken = 1;
            lk.unlock();
            const int st = be_->reset(r->cfg[0], r->key[0], r->ts[0]);
            lk.lock();
            r->status = st;
            r->left = 0;
            r->done = true;
            r->done_ns = steady_ns();
            st_.decided += 1;
            if (r->waiting) r->cv.notify_all();
            continue;
        }
        const int si = next_slot_;
        next_slot_ = (next_slot_ + 1) % (int)o_.max_in_flight;
        Slot& s = slots_[si];
        s.parts.clear();
        size_t m = 0;
        while (m < o_.max_batch && !queue_.empty() && !queue_.front()->reset_op) {
            Sub* sub = queue_.front();
            const size_t take = std::min(sub->m - sub->taken, (size_t)o_.max_batch - m);
            s.parts.push_back({sub, sub->taken, take, m});
            sub->taken += take;
            m += take;
            if (sub->taken == sub->m) queue_.pop_front();
        }
        pending_ -= m;
        inflight_++;
        lk.unlock();
        if (trace_cap_) s.t_form = steady_ns();
        // the submissions' inputs are immutable after Submit: copy unlocked
        for (const auto& p : s.parts) {
            memcpy(s.key + p.at, p.sub->key + p.off, 8 * p.count);
            memcpy(s.ts + p.at, p.sub->ts + p.off, 8 * p.count);
            memcpy(s.n + p.at, p.sub->n + p.off, 8 * p.count);
            memcpy(s.cfg + p.at, p.sub->cfg + p.off, 4 * p.count);
        }
        s.m = m;
        s.status = be_->launch(si, s);
        if (trace_cap_) s.t_launched = steady_ns();
        lk.lock();
        st_.batches++;
        st_.max_batch_seen = std::max<uint64_t>(st_.max_batch_seen, m);
        launched_.push_back(si);
        lk.unlock();
        cv_done_.notify_one();
    }
    std::lock_guard<std::mutex> g(mu_);
    sub_exited_ = true;
    cv_done_.notify_all();
}

void Coalescer::completer() {
    for (;;) {
        int si;
        {
            std::unique_lock<std::mutex> lk(mu_);
            cv_done_.wait(lk, [&] { return !launched_.empty() || sub_exited_; });
            if (launched_.empty()) break;
            si = launched_.front();
        }
        Slot& s = slots_[si];
        const int64_t t_wait = trace_cap_ ? steady_ns() : 0;
        int st = s.status == RL_OK ? be_->wait(si, s) : s.status;
        for (const auto& p : s.parts) {
            memcpy(p.sub->dec + p.off, s.dec + p.at, p.count);
            memcpy(p.sub->rem + p.off, s.rem + p.at, 8 * p.count);
            memcpy(p.sub->retry + p.off, s.retry + p.at, 8 * p.count);
            memcpy(p.sub->reset + p.off, s.reset + p.at, 8 * p.count);
        }
        const int64_t now = steady_ns();
        bool wake;
        {
            std::lock_guard<std::mutex> g(mu_);
            wake = sub_idle_;
            launched_.pop_front();
            inflight_--;
            if (trace_cap_) {
                BatchTrace t{done_batches_, s.m, 0, s.t_form, s.t_h2d, s.t_launched, t_wait, now};
                t.t_submit = s.parts.empty() ? s.t_form : s.parts[0].sub->submit_ns;   // the oldest request
                if (trace_.size() < trace_cap_) trace_.push_back(t);
                else trace_[done_batches_ % trace_cap_] = t;
            }
            done_batches_++;
            st_.decided += s.m;
            for (const auto& p : s.parts) {
                Sub* sub = p.sub;
                if (st != RL_OK) sub->status = st;
                sub->left -= p.count;
                if (sub->left == 0) {
                    sub->done = true;
                    sub->done_ns = now;
                    if (sub->waiting) sub->cv.notify_all();
                }
            }
        }
        if (wake) cv_sub_.notify_one();
    }
}

}  // namespace rlc

// ---------------------------------------------------------------------------
// C-ABI
// ---------------------------------------------------------------------------

struct rl_coalescer {
    rlc::Coalescer* c;
};

rlc::Coalescer* rlc::unwrap(rl_coalescer* c) { return c ? c->c : nullptr; }

static int create(std::unique_ptr<rlc::Backend> be, const rl_coalescer_opts* opts, rl_coalescer** out) {
    rl_coalescer_opts o{};
    if (opts) o = *opts;
    auto* c = new rlc::Coalescer(std::move(be), o);
    int rc = c->start();
    if (rc != RL_OK) {
        delete c;
        return rc;
    }
    *out = new rl_coalescer{c};
    return RL_OK;
}

extern "C" int rl_coalescer_create(rl_engine* e, const rl_coalescer_opts* opts, rl_coalescer** out) {
    if (!e || !out) return RL_EINVAL;
    return create(rlc::make_gpu_backend(e), opts, out);
}

extern "C" int rl_coalescer_create_with_backend(rl_batch_fn fn, void* user, const rl_coalescer_opts* opts,
                                                rl_coalescer** out) {
    if (!fn || !out) return RL_EINVAL;
    return create(rlc::make_fn_backend(fn, nullptr, user), opts, out);
}

extern "C" int rl_coalescer_create_with_backends(rl_batch_fn fn, rl_reset_fn reset_fn, void* user,
                                                 const rl_coalescer_opts* opts, rl_coalescer** out) {
    if (!fn || !out) return RL_EINVAL;
    return create(rlc::make_fn_backend(fn, reset_fn, user), opts, out);
}

extern "C" int rl_coalescer_reset(rl_coalescer* c, uint64_t key_id, int64_t ts_ns, uint32_t cfg_id) {
    if (!c) return RL_EINVAL;
    uint64_t t;
    const int64_t one = 1;
    int rc = c->c->Submit(1, &key_id, &ts_ns, &one, &cfg_id, &t, true);
    if (rc != RL_OK) return rc;
    return c->c->Wait(t, -1, nullptr, nullptr, nullptr, nullptr);
}

extern "C" int rl_coalescer_destroy(rl_coalescer* c) {
    if (!c) return RL_EINVAL;
    delete c->c;
    delete c;
    return RL_OK;
}

extern "C" int rl_coalescer_submit(rl_coalescer* c, size_t m, const uint64_t* key_id, const int64_t* ts_ns,
                                   const int64_t* n, const uint32_t* cfg_id, uint64_t* ticket) {
    if (!c) return RL_EINVAL;
    return c->c->Submit(m, key_id, ts_ns, n, cfg_id, ticket);
}

extern "C" int rl_coalescer_wait(rl_coalescer* c, uint64_t ticket, int64_t timeout_ns, uint8_t* decision,
                                 int64_t* remaining, int64_t* retry_after_ns, int64_t* reset_at_ns) {
    if (!c) return RL_EINVAL;
    return c->c->Wait(ticket, timeout_ns, decision, remaining, retry_after_ns, reset_at_ns);
}

extern "C" int rl_coalescer_decide(rl_coalescer* c, uint64_t key_id, int64_t ts_ns, int64_t n, uint32_t cfg_id,
                                   uint8_t* decision, int64_t* remaining, int64_t* retry_after_ns,
                                   int64_t* reset_at_ns) {
    if (!c) return RL_EINVAL;
    uint64_t t;
    int rc = c->c->Submit(1, &key_id, &ts_ns, &n, &cfg_id, &t);
    if (rc != RL_OK) return rc;
    return c->c->Wait(t, -1, decision, remaining, retry_after_ns, reset_at_ns);
}

extern "C" int rl_coalescer_get_stats(rl_coalescer* c, rl_coalescer_stats* out) {
    if (!c || !out) return RL_EINVAL;
    *out = c->c->Stats();
    return RL_OK;
}
