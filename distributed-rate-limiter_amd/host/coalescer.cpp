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
    op = OP_REQ;
    deadline = 0;
    done = waiting = cancelled = dropped = truncated = in_queue = waited = false;
    inflight = 0;
    done_ns = submit_ns = 0;
    tag = nullptr;
    now_ms = 0;
    cap_tb = cap_win = 0;
    info = rl_table_info{};
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
        if (m <= zero_copy_max_) {
            // zero-copy: the kernels read the requests from, and write the
            // results into, the pinned slot itself (host memory the device
            // maps).  No hipMemcpyAsync on the submit path: the configs[4]
            // stalls were the submitter blocked ~8 ms inside those calls
            // with the device idle (profiles/r3d_stall_trace.json)
            s.t_h2d = steady_ns();
            int rc = rl_decide_batch_device(e_, m, s.key, s.ts, s.n, s.cfg, nullptr, s.dec, s.rem, s.retry, s.reset,
                                            nullptr, os_);
            if (rc != RL_OK) return rc;
            return hipEventRecord(d.ev, os_) == hipSuccess ? RL_OK : RL_EDEVICE;
        }
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
    int launch_reset(int i, Slot& s, uint32_t cfg, uint64_t key, int64_t ts) override {
        (void)hipSetDevice(dev_id_);   // the submitter thread
        s.t_h2d = steady_ns();
        // enqueued on the engine's replay stream between two batches; the
        // output stream (and so this slot's completion event) waits for it
        const int rc = rl_reset_device(e_, cfg, key, ts, os_);
        if (rc != RL_OK) return rc;
        return hipEventRecord(dev_[i].ev, os_) == hipSuccess ? RL_OK : RL_EDEVICE;
    }
    int wait(int i, Slot&) override {
        (void)hipSetDevice(dev_id_);   // the completer thread
        return await_event(dev_[i].ev) == hipSuccess ? RL_OK : RL_EDEVICE;
    }
    int table_info(int64_t now_ms, rl_table_info* out) override {
        (void)hipSetDevice(dev_id_);
        return rl_table_info_get(e_, now_ms, out);
    }
    int gc(int64_t now_ms, uint64_t tb_cap, uint64_t win_cap, rl_table_info* out) override {
        (void)hipSetDevice(dev_id_);
        return rl_table_gc(e_, now_ms, tb_cap, win_cap, out);
    }
    int table_of(uint32_t cfg) override {
        if (cfg >= table_.size()) {      // configs registered since: look them up once
            for (uint32_t c = (uint32_t)table_.size();; c++) {
                const int t = rl_config_table(e_, c);
                if (t < 0) break;
                table_.push_back((int8_t)t);
            }
        }
        return cfg < table_.size() ? table_[cfg] : -1;
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
    std::vector<int8_t> table_;  // table_of per config id (submitter thread)
    int dev_id_ = 0;             // the engine's device: current when the coalescer is created
    // batches up to this size run zero-copy on the pinned slot (larger ones:
    // one H2D copy, device-resident inputs for the grouping's several reads)
    size_t zero_copy_max_ = getenv("RL_COALESCER_ZC_MAX") ? strtoull(getenv("RL_COALESCER_ZC_MAX"), nullptr, 10)
                                                          : (size_t)65536;
    hipStream_t cs_ = nullptr, os_ = nullptr;
    std::vector<void*> host_;
    std::vector<Dev> dev_;
    size_t M_ = 0;
};

// synchronous host functions (the CPU tests plug the oracle in here)
class FnBackend : public Backend {
public:
    explicit FnBackend(const rl_coalescer_backend& b) : b_(b) {}
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
        return b_.batch(b_.user, s.m, s.key, s.ts, s.n, s.cfg, s.dec, s.rem, s.retry, s.reset);
    }
    int launch_reset(int, Slot& s, uint32_t cfg, uint64_t key, int64_t ts) override {
        s.t_h2d = steady_ns();
        return b_.reset ? b_.reset(b_.user, cfg, key, ts) : RL_EINVAL;
    }
    int wait(int, Slot&) override { return RL_OK; }
    int table_info(int64_t now_ms, rl_table_info* out) override {
        return b_.table_info ? b_.table_info(b_.user, now_ms, out) : RL_EINVAL;
    }
    int gc(int64_t now_ms, uint64_t tb_cap, uint64_t win_cap, rl_table_info* out) override {
        return b_.gc ? b_.gc(b_.user, now_ms, tb_cap, win_cap, out) : RL_EINVAL;
    }

private:
    rl_coalescer_backend b_;
    std::vector<std::unique_ptr<uint8_t[]>> mem_;
};

std::unique_ptr<Backend> make_gpu_backend(rl_engine* e) { return std::unique_ptr<Backend>(new GpuBackend(e)); }
std::unique_ptr<Backend> make_fn_backend(const rl_coalescer_backend& b) {
    return std::unique_ptr<Backend>(new FnBackend(b));
}

// ---------------------------------------------------------------------------


Coalescer::Coalescer(std::unique_ptr<Backend> be, const rl_coalescer_opts& o) : be_(std::move(be)), o_(o) {
    if (o_.max_batch == 0) o_.max_batch = 65536;
    if (o_.max_in_flight == 0) o_.max_in_flight = 3;
    if (o_.max_in_flight > 3) o_.max_in_flight = 3;
    if (o_.queue_cap == 0) o_.queue_cap = 1ull << 24;
    if (o_.linger_ns < 0) o_.linger_ns = 0;
    if (o_.gc_high_pct == 0 || o_.gc_high_pct > 95) o_.gc_high_pct = 50;
    if (o_.gc_margin_ms <= 0) o_.gc_margin_ms = 1000;
    if (o_.gc_interval_ns < 0) o_.gc_interval_ns = 0;
    if (const char* v = getenv("RL_COALESCER_TRACE")) trace_cap_ = (size_t)strtoull(v, nullptr, 10);
    st_.struct_size = sizeof(rl_coalescer_stats);
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
            notify_locked(s);
        }
    }
}

void Coalescer::SetNotify(NotifyFn fn, void* user) {
    std::lock_guard<std::mutex> g(mu_);
    notify_ = fn;
    notify_user_ = user;
}

int Coalescer::Submit(size_t m, const uint64_t* key, const int64_t* ts, const int64_t* n, const uint32_t* cfg,
                      uint64_t* ticket, int64_t deadline, void* tag) {
    if (!ticket || (m && (!key || !ts || !n || !cfg)) || deadline < 0) return RL_EINVAL;
    Sub* s = get_sub(m);
    s->deadline = deadline;
    s->tag = tag;
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
            s->in_queue = true;
            pending_ += m;
        } else {
            s->done = true;
            s->done_ns = steady_ns();
            notify_locked(s);
        }
        *ticket = s->first;
        // wake the submitter only when it sleeps: at millions of submissions
        // per second an unconditional notify is a futex call per submission
        if (!m || !sub_idle_) return RL_OK;
    }
    cv_sub_.notify_one();
    return RL_OK;
}

int Coalescer::SubmitOp(Op op, uint64_t key, int64_t ts, uint32_t cfg, int64_t now_ms, uint64_t cap_tb,
                        uint64_t cap_win, uint64_t* ticket, void* tag) {
    Sub* s = get_sub(1);
    s->op = op;
    s->tag = tag;
    s->key[0] = key;
    s->ts[0] = ts;
    s->n[0] = 1;
    s->cfg[0] = cfg;
    s->now_ms = now_ms;
    s->cap_tb = cap_tb;
    s->cap_win = cap_win;
    if (trace_cap_) s->submit_ns = steady_ns();
    {
        std::lock_guard<std::mutex> g(mu_);
        if (stop_) {
            put_sub(s);
            return RL_ECLOSED;
        }
        s->first = next_seq_++;
        subs_[s->first] = s;
        queue_.push_back(s);
        s->in_queue = true;
        pending_ += 1;
        *ticket = s->first;
        if (!sub_idle_) return RL_OK;
    }
    cv_sub_.notify_one();
    return RL_OK;
}

void Coalescer::drop_locked(Sub* s, int code) {
    // none of it was launched: every request is still pending
    pending_ -= s->m - s->taken;
    if (s->op == OP_REQ) (code == RL_ECANCELED ? st_.cancelled : st_.expired) += s->m;
    s->dropped = true;
    s->done = true;
    s->status = code;
    s->left = 0;
    s->done_ns = steady_ns();
    if (s->waiting) s->cv.notify_all();
    notify_locked(s);
}

void Coalescer::truncate_locked(Sub* s, int code) {
    // part of it was launched (applied, as an EVAL already sent); the part not
    // yet launched is dropped unapplied, so nothing is sent after its context
    // ended.  taken = m stops the submitter; it pops the submission when it
    // reaches the head of the queue
    const size_t rest = s->m - s->taken;
    if (rest == 0) return;
    // the outcome is the context's error, whoever completes it: the results
    // of the launched part are discarded and the tail never ran (its result
    // arrays hold whatever a pooled Sub held before)
    s->truncated = true;
    s->status = code;
    pending_ -= rest;
    if (s->op == OP_REQ) (code == RL_ECANCELED ? st_.cancelled : st_.expired) += rest;
    s->taken = s->m;
    s->left -= rest;
    if (s->left == 0 && !s->done) {
        s->done = true;
        s->done_ns = steady_ns();
        if (s->waiting) s->cv.notify_all();
        notify_locked(s);
    }
}

void Coalescer::maybe_free_locked(Sub* s) {
    if (s->waited && !s->in_queue && s->inflight == 0) put_sub(s);
}

int Coalescer::Cancel(uint64_t ticket) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = subs_.find(ticket);
    if (it == subs_.end()) return RL_EINVAL;
    Sub* s = it->second;
    if (s->done) return RL_OK;
    s->cancelled = true;
    if (s->taken == 0) drop_locked(s, RL_ECANCELED);
    else {
        truncate_locked(s, RL_ECANCELED);
        if (s->waiting) s->cv.notify_all();
    }
    return RL_OK;
}

int Coalescer::Wait(uint64_t ticket, int64_t timeout_ns, uint8_t* dec, int64_t* rem, int64_t* retry,
                    int64_t* reset, int64_t* done_ns, rl_table_info* info) {
    std::unique_lock<std::mutex> lk(mu_);
    auto it = subs_.find(ticket);
    if (it == subs_.end()) return RL_EINVAL;
    Sub* s = it->second;
    const int64_t t_end = timeout_ns < 0 ? INT64_MAX : steady_ns() + timeout_ns;
    int code = RL_OK;   // != RL_OK: the ticket ends without results
    for (;;) {
        if (s->cancelled) { code = RL_ECANCELED; break; }
        if (s->done) {
            if (s->dropped || s->truncated) code = s->status;
            break;
        }
        const int64_t now = steady_ns();
        if (s->deadline && now >= s->deadline) {
            // not launched: never applied; launched: applied, results discarded,
            // and what was not launched yet never will be
            if (s->taken == 0) drop_locked(s, RL_EDEADLINE);
            else truncate_locked(s, RL_EDEADLINE);
            code = RL_EDEADLINE;
            break;
        }
        if (now >= t_end) {
            s->waiting = false;
            return RL_ETIMEOUT;
        }
        s->waiting = true;
        const int64_t until = s->deadline ? std::min(t_end, s->deadline) : t_end;
        if (until == INT64_MAX) s->cv.wait(lk);
        else s->cv.wait_for(lk, std::chrono::nanoseconds(until - now));
    }
    s->waiting = false;
    subs_.erase(it);
    if (code != RL_OK) {
        if (done_ns) *done_ns = steady_ns();
        s->waited = true;
        maybe_free_locked(s);
        return code;
    }
    // done and applied: no slot or queue references it any more
    lk.unlock();
    const size_t m = s->m;
    if (s->op == OP_REQ) {
        if (dec) memcpy(dec, s->dec, m);
        if (rem) memcpy(rem, s->rem, 8 * m);
        if (retry) memcpy(retry, s->retry, 8 * m);
        if (reset) memcpy(reset, s->reset, 8 * m);
    }
    if (info) *info = s->info;
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
    if (trace_cap_ == 0 || trace_.size() < trace_cap_) return trace_;
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

int Coalescer::run_table_op(Sub* op) {
    rl_table_info info{};
    info.struct_size = sizeof info;
    int st;
    if (op->op == OP_INFO) {
        st = be_->table_info(op->now_ms, &info);
    } else {
        st = be_->gc(op->now_ms, op->cap_tb, op->cap_win, &info);
        std::lock_guard<std::mutex> g(mu_);
        st_.gc_runs++;
        if (st != RL_OK) st_.gc_failures++;
    }
    op->info = info;
    return st;
}

// Automatic GC (include/rl_coalescer.h, rl_coalescer_opts.gc_*): every request
// inserts at most one entry into one table (a window request may also move one
// window key to the spill table), so after a count with `budget` free slots
// below the high-water mark of the fullest table, that many requests cannot
// push any table past it.  Runs before launching `s`, so a GC lands between
// the batches launched before and `s`.
void Coalescer::auto_gc(const Slot& s) {
    if (o_.gc_interval_ns <= 0 || s.m == 0) return;
    const int64_t now = steady_ns();
    // the batch's requests per table: a token-bucket request can insert one
    // entry into the token-bucket table, a window request one into the window
    // table and one into the spill table; a request of an unknown config counts
    // for both
    uint64_t mt[2] = {0, 0};
    for (size_t i = 0; i < s.m; i++) {
        const int t = be_->table_of(s.cfg[i]);
        if (t != 1) mt[0]++;
        if (t != 0) mt[1]++;
    }
    if (gc_counted_ && gc_launched_[0] + mt[0] <= gc_budget_[0] && gc_launched_[1] + mt[1] <= gc_budget_[1] &&
        now - gc_last_check_ < o_.gc_interval_ns) {
        gc_launched_[0] += mt[0];
        gc_launched_[1] += mt[1];
        return;
    }
    // server clock of the GC: no later request may carry an older one (the
    // engine's clock is floor(ts / 1e6)); requests come in near time order,
    // within gc_margin_ms of each other
    int64_t min_ts = INT64_MAX;
    for (size_t i = 0; i < s.m; i++) min_ts = std::min(min_ts, s.ts[i]);
    const int64_t now_ms = (min_ts >= 0 ? min_ts / 1000000 : -((-min_ts + 999999) / 1000000)) - o_.gc_margin_ms;
    rl_table_info in{};
    in.struct_size = sizeof in;
    if (be_->table_info(now_ms, &in) != RL_OK) {
        gc_counted_ = true;
        gc_budget_[0] = gc_budget_[1] = 0;
        gc_last_check_ = now;
        gc_launched_[0] = mt[0];
        gc_launched_[1] = mt[1];
        return;
    }
    const double hi = o_.gc_high_pct / 100.0;
    auto high = [&](uint64_t cap) { return (uint64_t)(hi * (double)cap); };
    auto full = [&](uint64_t used, uint64_t cap, uint64_t m) { return used + m > high(cap); };
    {
        std::lock_guard<std::mutex> g(mu_);
        st_.gc_checks++;
    }
    if (full(in.tb_used, in.tb_capacity, mt[0]) || full(in.win_used, in.win_capacity, mt[1]) ||
        full(in.spill_used, in.spill_capacity, mt[1])) {
        // grow a table whose live keys alone fill half its headroom
        auto grow = [&](uint64_t live, uint64_t cap, uint64_t lim) -> uint64_t {
            if (live <= high(cap) / 2) return 0;
            if (lim && 2 * cap > lim) return 0;
            return 2 * cap;
        };
        const uint64_t ntb = grow(in.tb_live, in.tb_capacity, o_.gc_max_tb_capacity);
        uint64_t nwin = grow(in.win_live, in.win_capacity, o_.gc_max_win_capacity);
        if (!nwin && in.spill_live > high(in.spill_capacity) / 2 &&
            !(o_.gc_max_win_capacity && 2 * in.win_capacity > o_.gc_max_win_capacity))
            nwin = 2 * in.win_capacity;   // the spill table follows the window table
        rl_table_info out{};
        out.struct_size = sizeof out;
        int st = be_->gc(now_ms, ntb, nwin, &out);
        bool ok = st == RL_OK;
        if (!ok && (ntb || nwin)) ok = be_->gc(now_ms, 0, 0, &out) == RL_OK;   // no room to grow: in place
        {
            std::lock_guard<std::mutex> g(mu_);
            st_.gc_runs++;
            if (!ok) st_.gc_failures++;
        }
        if (ok) in = out;
    }
    auto room = [&](uint64_t used, uint64_t cap) -> uint64_t { return used < high(cap) ? high(cap) - used : 0; };
    gc_budget_[0] = room(in.tb_used, in.tb_capacity);
    gc_budget_[1] = std::min(room(in.win_used, in.win_capacity), room(in.spill_used, in.spill_capacity));
    gc_counted_ = true;
    gc_last_check_ = now;
    gc_launched_[0] = mt[0];      // this batch launches after the count
    gc_launched_[1] = mt[1];
}

void Coalescer::submitter() {
    for (;;) {
        std::unique_lock<std::mutex> lk(mu_);
        sub_idle_ = true;
        cv_sub_.wait(lk, [&] { return (stop_ && pending_ == 0) || (pending_ > 0 && inflight_ < (int)o_.max_in_flight); });
        sub_idle_ = false;
        if (pending_ == 0) break;   // stop_ with nothing left
        // submissions dropped while queued (deadline, cancel) leave the queue here
        auto pop_dropped = [&] {
            while (!queue_.empty() && queue_.front()->dropped) {
                Sub* d = queue_.front();
                queue_.pop_front();
                d->in_queue = false;
                maybe_free_locked(d);
            }
        };
        pop_dropped();
        if (o_.linger_ns > 0 && inflight_ == 0 && pending_ < o_.max_batch && !stop_ && queue_.front()->op == OP_REQ) {
            const auto until = std::chrono::steady_clock::now() + std::chrono::nanoseconds(o_.linger_ns);
            sub_idle_ = true;
            cv_sub_.wait_until(lk, until, [&] { return stop_ || pending_ >= o_.max_batch; });
            sub_idle_ = false;
            pop_dropped();
            if (pending_ == 0) continue;
        }
        Sub* f = queue_.front();
        if (f->op == OP_INFO || f->op == OP_GC) {
            // synchronous, on this thread: every batch before it is launched
            // and the backend drains them; nothing after it is launched yet
            queue_.pop_front();
            f->in_queue = false;
            pending_ -= 1;
            f->taken = 1;
            lk.unlock();
            const int st = run_table_op(f);
            lk.lock();
            f->status = st;
            f->left = 0;
            f->done = true;
            f->done_ns = steady_ns();
            if (f->waiting) f->cv.notify_all();
            notify_locked(f);
            maybe_free_locked(f);
            // a manual GC invalidates the automatic GC's count
            gc_counted_ = false;
            continue;
        }
        const int si = next_slot_;
        Slot& s = slots_[si];
        s.parts.clear();
        s.is_reset = false;
        size_t m = 0;
        if (f->op == OP_RESET) {
            // like a one-request batch: enqueued between the batches around it
            queue_.pop_front();
            f->in_queue = false;
            f->taken = 1;
            f->inflight = 1;
            pending_ -= 1;
            s.parts.push_back({f, 0, 1, 0});
            s.is_reset = true;
        } else {
            const int64_t now = steady_ns();
            while (m < o_.max_batch && !queue_.empty()) {
                Sub* sub = queue_.front();
                if (sub->dropped) {
                    queue_.pop_front();
                    sub->in_queue = false;
                    maybe_free_locked(sub);
                    continue;
                }
                if (sub->op != OP_REQ) break;
                if (sub->taken < sub->m && (sub->cancelled || (sub->deadline && sub->deadline <= now))) {
                    // its context ended before (the rest of) it was sent: that part is never applied
                    if (sub->taken == 0) drop_locked(sub, sub->cancelled ? RL_ECANCELED : RL_EDEADLINE);
                    else truncate_locked(sub, sub->cancelled ? RL_ECANCELED : RL_EDEADLINE);
                }
                if (sub->dropped || sub->taken == sub->m) {
                    // dropped, or the rest of a split submission truncated: nothing left to launch
                    queue_.pop_front();
                    sub->in_queue = false;
                    maybe_free_locked(sub);
                    continue;
                }
                const size_t take = std::min(sub->m - sub->taken, (size_t)o_.max_batch - m);
                s.parts.push_back({sub, sub->taken, take, m});
                sub->taken += take;
                sub->inflight++;
                m += take;
                if (sub->taken == sub->m) {
                    queue_.pop_front();
                    sub->in_queue = false;
                }
            }
            if (m == 0) continue;   // everything at the head was dropped
            pending_ -= m;
        }
        next_slot_ = (next_slot_ + 1) % (int)o_.max_in_flight;
        inflight_++;
        lk.unlock();
        if (trace_cap_) s.t_form = steady_ns();
        if (s.is_reset) {
            const Sub* r = s.parts[0].sub;
            s.m = 0;
            s.status = be_->launch_reset(si, s, r->cfg[0], r->key[0], r->ts[0]);
        } else {
            // the submissions' inputs are immutable after Submit: copy unlocked
            for (const auto& p : s.parts) {
                memcpy(s.key + p.at, p.sub->key + p.off, 8 * p.count);
                memcpy(s.ts + p.at, p.sub->ts + p.off, 8 * p.count);
                memcpy(s.n + p.at, p.sub->n + p.off, 8 * p.count);
                memcpy(s.cfg + p.at, p.sub->cfg + p.off, 4 * p.count);
            }
            s.m = m;
            auto_gc(s);
            s.status = be_->launch(si, s);
        }
        if (trace_cap_) s.t_launched = steady_ns();
        lk.lock();
        st_.batches++;
        st_.max_batch_seen = std::max<uint64_t>(st_.max_batch_seen, m);
        launched_.push_back(si);
        lk.unlock();
        cv_done_.notify_one();
    }
    std::lock_guard<std::mutex> g(mu_);
    // only dropped submissions can be left in the queue
    while (!queue_.empty()) {
        Sub* d = queue_.front();
        queue_.pop_front();
        d->in_queue = false;
        maybe_free_locked(d);
    }
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
        if (!s.is_reset) {
            for (const auto& p : s.parts) {
                memcpy(p.sub->dec + p.off, s.dec + p.at, p.count);
                memcpy(p.sub->rem + p.off, s.rem + p.at, 8 * p.count);
                memcpy(p.sub->retry + p.off, s.retry + p.at, 8 * p.count);
                memcpy(p.sub->reset + p.off, s.reset + p.at, 8 * p.count);
            }
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
            st_.decided += s.is_reset ? 1 : s.m;
            for (const auto& p : s.parts) {
                Sub* sub = p.sub;
                if (st != RL_OK && !sub->truncated) sub->status = st;
                sub->left -= p.count;
                sub->inflight--;
                if (sub->left == 0 && !sub->done) {
                    sub->done = true;
                    sub->done_ns = now;
                    if (sub->waiting) sub->cv.notify_all();
                    notify_locked(sub);
                }
                maybe_free_locked(sub);   // orphaned (its waiter gave up) and now complete
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
    if (!out) return RL_EINVAL;
    rl_coalescer_opts o{};
    o.struct_size = sizeof o;
    if (opts) {
        if (opts->struct_size != sizeof(rl_coalescer_opts)) return RL_EINVAL;
        o = *opts;
    }
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

extern "C" int rl_coalescer_create_with_host_backend(const rl_coalescer_backend* be, const rl_coalescer_opts* opts,
                                                     rl_coalescer** out) {
    if (!be || be->struct_size != sizeof(rl_coalescer_backend) || !be->batch || !out) return RL_EINVAL;
    return create(rlc::make_fn_backend(*be), opts, out);
}

extern "C" int rl_coalescer_create_with_backend(rl_batch_fn fn, void* user, const rl_coalescer_opts* opts,
                                                rl_coalescer** out) {
    return rl_coalescer_create_with_backends(fn, nullptr, user, opts, out);
}

extern "C" int rl_coalescer_create_with_backends(rl_batch_fn fn, rl_reset_fn reset_fn, void* user,
                                                 const rl_coalescer_opts* opts, rl_coalescer** out) {
    rl_coalescer_backend b{sizeof(rl_coalescer_backend), fn, reset_fn, nullptr, nullptr, user};
    return rl_coalescer_create_with_host_backend(&b, opts, out);
}

extern "C" int rl_coalescer_destroy(rl_coalescer* c) {
    if (!c) return RL_EINVAL;
    delete c->c;
    delete c;
    return RL_OK;
}

extern "C" int64_t rl_coalescer_now_ns(void) { return rlc::steady_ns(); }

extern "C" int rl_coalescer_submit(rl_coalescer* c, size_t m, const uint64_t* key_id, const int64_t* ts_ns,
                                   const int64_t* n, const uint32_t* cfg_id, uint64_t* ticket) {
    if (!c) return RL_EINVAL;
    return c->c->Submit(m, key_id, ts_ns, n, cfg_id, ticket);
}

extern "C" int rl_coalescer_submit_deadline(rl_coalescer* c, size_t m, const uint64_t* key_id, const int64_t* ts_ns,
                                            const int64_t* n, const uint32_t* cfg_id, int64_t deadline_ns,
                                            uint64_t* ticket) {
    if (!c) return RL_EINVAL;
    return c->c->Submit(m, key_id, ts_ns, n, cfg_id, ticket, deadline_ns);
}

extern "C" int rl_coalescer_cancel(rl_coalescer* c, uint64_t ticket) {
    if (!c) return RL_EINVAL;
    return c->c->Cancel(ticket);
}

extern "C" int rl_coalescer_wait(rl_coalescer* c, uint64_t ticket, int64_t timeout_ns, uint8_t* decision,
                                 int64_t* remaining, int64_t* retry_after_ns, int64_t* reset_at_ns) {
    if (!c) return RL_EINVAL;
    return c->c->Wait(ticket, timeout_ns, decision, remaining, retry_after_ns, reset_at_ns);
}

extern "C" int rl_coalescer_decide(rl_coalescer* c, uint64_t key_id, int64_t ts_ns, int64_t n, uint32_t cfg_id,
                                   uint8_t* decision, int64_t* remaining, int64_t* retry_after_ns,
                                   int64_t* reset_at_ns) {
    return rl_coalescer_decide_deadline(c, key_id, ts_ns, n, cfg_id, 0, decision, remaining, retry_after_ns,
                                        reset_at_ns);
}

extern "C" int rl_coalescer_decide_deadline(rl_coalescer* c, uint64_t key_id, int64_t ts_ns, int64_t n,
                                            uint32_t cfg_id, int64_t deadline_ns, uint8_t* decision,
                                            int64_t* remaining, int64_t* retry_after_ns, int64_t* reset_at_ns) {
    if (!c) return RL_EINVAL;
    uint64_t t;
    int rc = c->c->Submit(1, &key_id, &ts_ns, &n, &cfg_id, &t, deadline_ns);
    if (rc != RL_OK) return rc;
    return c->c->Wait(t, -1, decision, remaining, retry_after_ns, reset_at_ns);
}

extern "C" int rl_coalescer_reset(rl_coalescer* c, uint64_t key_id, int64_t ts_ns, uint32_t cfg_id) {
    if (!c) return RL_EINVAL;
    uint64_t t;
    int rc = c->c->SubmitOp(rlc::OP_RESET, key_id, ts_ns, cfg_id, 0, 0, 0, &t);
    if (rc != RL_OK) return rc;
    return c->c->Wait(t, -1, nullptr, nullptr, nullptr, nullptr);
}

static int table_op(rl_coalescer* c, rlc::Op op, int64_t now_ms, uint64_t tb, uint64_t win, rl_table_info* out) {
    uint64_t t;
    int rc = c->c->SubmitOp(op, 0, 0, 0, now_ms, tb, win, &t);
    if (rc != RL_OK) return rc;
    rl_table_info info{};
    rc = c->c->Wait(t, -1, nullptr, nullptr, nullptr, nullptr, nullptr, &info);
    if (out && rc == RL_OK) {
        const uint32_t n = (uint32_t)std::min<size_t>(out->struct_size, sizeof info);   // bytes filled in
        info.struct_size = n;
        memcpy(out, &info, n);
    }
    return rc;
}

extern "C" int rl_coalescer_table_info(rl_coalescer* c, int64_t now_ms, rl_table_info* out) {
    if (!c || !out || out->struct_size < 8) return RL_EINVAL;
    return table_op(c, rlc::OP_INFO, now_ms, 0, 0, out);
}

extern "C" int rl_coalescer_gc(rl_coalescer* c, int64_t now_ms, uint64_t tb_capacity, uint64_t win_capacity,
                               rl_table_info* out) {
    if (!c || (out && out->struct_size < 8)) return RL_EINVAL;
    return table_op(c, rlc::OP_GC, now_ms, tb_capacity, win_capacity, out);
}

extern "C" int rl_coalescer_get_stats(rl_coalescer* c, rl_coalescer_stats* out) {
    if (!c || !out || out->struct_size < 8) return RL_EINVAL;
    rl_coalescer_stats s = c->c->Stats();
    const uint32_t n = (uint32_t)std::min<size_t>(out->struct_size, sizeof s);   // bytes filled in
    s.struct_size = n;
    memcpy(out, &s, n);
    return RL_OK;
}
