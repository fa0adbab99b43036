// coalescer.hpp -- request coalescer in front of the decision engine
// (include/rl_coalescer.h has the policy, ordering and context contract).
//
// The reference's Limiter.AllowN is one Redis EVAL per call
// (tokenbucket.go:172, slidingwindow.go:164, fixedwindow.go:152); the north
// star's BatchAllow path gathers concurrent calls into GPU batches
// (SURVEY.md §8b, §8f rank 1).  Threads: callers submit and wait; one
// submitter thread forms batches and launches them (and runs the ordered
// table operations); one completer thread waits for each launch in order and
// hands results back.
#pragma once

#include <stdint.h>

#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/rl_coalescer.h"

namespace rlc {

// one launch's staging buffers (host side; pinned for the GPU backend)
struct Slot {
    uint64_t* key = nullptr;
    int64_t* ts = nullptr;
    int64_t* n = nullptr;
    uint32_t* cfg = nullptr;
    uint8_t* dec = nullptr;
    int64_t* rem = nullptr;
    int64_t* retry = nullptr;
    int64_t* reset = nullptr;
    size_t m = 0;
    bool is_reset = false;   // a Reset (parts[0].sub), not requests
    int status = RL_OK;
    int64_t t_form = 0, t_h2d = 0, t_launched = 0;   // steady ns (batch trace)
    struct Part {
        struct Sub* sub;
        size_t off, count, at;   // sub[off, off+count) <-> slot[at, at+count)
    };
    std::vector<Part> parts;
};

// where batches go: the GPU engine, or synchronous host functions (tests)
class Backend {
public:
    virtual ~Backend() = default;
    virtual int init(int nslots, size_t max_batch, std::vector<Slot>* slots) = 0;
    virtual int launch(int slot, Slot& s) = 0;   // asynchronous
    // Reset after every launched batch and before every later one,
    // asynchronous like a launch (completes through wait(slot))
    virtual int launch_reset(int slot, Slot& s, uint32_t cfg, uint64_t key, int64_t ts) = 0;
    virtual int wait(int slot, Slot& s) = 0;     // until launch `slot` completed
    // synchronous table operations (the GPU engine drains its batches first)
    virtual int table_info(int64_t now_ms, rl_table_info* out) = 0;
    virtual int gc(int64_t now_ms, uint64_t tb_cap, uint64_t win_cap, rl_table_info* out) = 0;
    // the table a config's keys live in (0 token bucket, 1 window), or -1
    // when unknown (the automatic GC then counts the request against both)
    virtual int table_of(uint32_t cfg) { (void)cfg; return -1; }
};

std::unique_ptr<Backend> make_gpu_backend(rl_engine* e);
std::unique_ptr<Backend> make_fn_backend(const rl_coalescer_backend& b);

enum Op : uint8_t { OP_REQ, OP_RESET, OP_INFO, OP_GC };

// one submission: its requests (copied) and results, or one table operation
struct Sub {
    uint64_t first = 0;
    size_t m = 0, taken = 0, left = 0;
    int status = RL_OK;
    Op op = OP_REQ;
    int64_t deadline = 0;         // steady ns; 0 = none
    bool done = false;
    bool waiting = false;         // a caller blocks on cv (else completion skips the wake)
    bool cancelled = false;       // rl_coalescer_cancel before completion
    bool dropped = false;         // completed unapplied (deadline / cancel before launch)
    bool truncated = false;       // launched in part; the rest dropped (deadline / cancel): no results
    bool in_queue = false;        // queue_ still holds it (the submitter pops it)
    bool waited = false;          // the caller released its ticket
    uint32_t inflight = 0;        // slot parts launched, not completed
    int64_t done_ns = 0;          // steady clock at completion
    int64_t submit_ns = 0;        // steady clock at Submit (batch trace)
    void* tag = nullptr;          // the caller's completion tag (SetNotify)
    // OP_INFO / OP_GC arguments and result
    int64_t now_ms = 0;
    uint64_t cap_tb = 0, cap_win = 0;
    rl_table_info info{};
    std::condition_variable cv;
    std::unique_ptr<uint8_t[]> mem;
    uint64_t* key;
    int64_t *ts, *n, *rem, *retry, *reset;
    uint32_t* cfg;
    uint8_t* dec;
    size_t cap = 0;               // requests the buffer holds (pooled Subs are reused)
    explicit Sub(size_t m);
    void carve(size_t m);         // reset for a new submission of m <= cap requests
};

int64_t steady_ns();

// One launched batch, for stall attribution (RL_COALESCER_TRACE=<ring size>):
// steady-clock ns of the oldest request's Submit, the batch taken from the
// queue, inputs on the device (H2D done), the engine call returned, the
// completer starting to wait, and the results back on the host.
struct BatchTrace {
    uint64_t seq;
    uint64_t m;
    int64_t t_submit, t_form, t_h2d, t_launched, t_wait, t_done;
};

class Coalescer {
public:
    Coalescer(std::unique_ptr<Backend> be, const rl_coalescer_opts& o);
    ~Coalescer();
    int start();
    // tag: with SetNotify, the completion callback receives it
    int Submit(size_t m, const uint64_t* key, const int64_t* ts, const int64_t* n, const uint32_t* cfg,
               uint64_t* ticket, int64_t deadline = 0, void* tag = nullptr);
    // a Reset / table count / table GC, queued in sequence order
    int SubmitOp(Op op, uint64_t key, int64_t ts, uint32_t cfg, int64_t now_ms, uint64_t cap_tb,
                 uint64_t cap_win, uint64_t* ticket, void* tag = nullptr);
    // Completion callback for submissions made with a tag: fn(user, ticket,
    // tag) runs once when the submission is done (applied, failed, or dropped
    // unapplied), on a coalescer thread (or the thread of a Cancel / Wait that
    // dropped it) WITH THE COALESCER LOCK HELD: it must only hand the ticket
    // to its owner (an event loop then collects it with Wait(ticket, 0, ...))
    // and never call back into the coalescer.  Set before the first tagged
    // submission.
    using NotifyFn = void (*)(void* user, uint64_t ticket, void* tag);
    void SetNotify(NotifyFn fn, void* user);
    int Cancel(uint64_t ticket);
    // done_ns (optional): steady-clock completion time of the submission;
    // info (optional): an OP_INFO / OP_GC result
    int Wait(uint64_t ticket, int64_t timeout_ns, uint8_t* dec, int64_t* rem, int64_t* retry, int64_t* reset,
             int64_t* done_ns = nullptr, rl_table_info* info = nullptr);
    rl_coalescer_stats Stats();
    void Shutdown();
    // the trace ring, oldest first (empty unless RL_COALESCER_TRACE is set)
    std::vector<BatchTrace> Trace();

private:
    void submitter();
    void completer();
    // drop a submission none of whose requests was launched: done, unapplied
    void drop_locked(Sub* s, int code);
    // a submission split across launches whose context ended: drop the part
    // not launched yet (never applied); the launched part completes as usual
    void truncate_locked(Sub* s, int code);
    // a submission became done (lock held): the completion callback
    void notify_locked(Sub* s) {
        if (notify_ && s->tag) notify_(notify_user_, s->first, s->tag);
    }
    NotifyFn notify_ = nullptr;
    void* notify_user_ = nullptr;
    // free a submission no one references any more (queue, slots, caller)
    void maybe_free_locked(Sub* s);
    // automatic GC before launching `s` (submitter thread, lock not held)
    void auto_gc(const Slot& s);
    // run a synchronous table operation (submitter thread, lock not held)
    int run_table_op(Sub* op);
    // pooled submissions: no heap allocation (and no mmap / page faults for
    // large ones) per Submit in steady state
    Sub* get_sub(size_t m);
    void put_sub(Sub* s);
    std::mutex pool_mu_;
    std::vector<Sub*> pool_;

    std::unique_ptr<Backend> be_;
    rl_coalescer_opts o_;
    std::vector<Slot> slots_;
    std::mutex mu_;
    std::condition_variable cv_sub_, cv_done_, cv_space_;
    std::deque<Sub*> queue_;                       // submissions with requests not yet launched
    std::unordered_map<uint64_t, Sub*> subs_;      // by ticket, until waited for
    std::deque<int> launched_;                     // slots on the device, in launch order
    uint64_t next_seq_ = 0, pending_ = 0;
    int inflight_ = 0, next_slot_ = 0;
    bool stop_ = false, sub_exited_ = false;
    bool sub_idle_ = false;        // the submitter sleeps on cv_sub_ (submit wakes it only then)
    rl_coalescer_stats st_{};
    std::vector<BatchTrace> trace_;   // ring of trace_cap_ batches
    size_t trace_cap_ = 0;
    uint64_t done_batches_ = 0;
    // automatic GC (submitter thread only)
    int64_t gc_last_check_ = 0;       // steady ns
    // requests launched since the last count that may insert into the
    // token-bucket table [0] / the window and spill tables [1], and how many
    // cannot fill them past gc_high_pct
    uint64_t gc_launched_[2] = {0, 0};
    uint64_t gc_budget_[2] = {0, 0};
    bool gc_counted_ = false;         // a first count was taken
    std::thread t_sub_, t_done_;
};

// the C++ object behind a C-ABI handle (bench_e2e reads completion times)
Coalescer* unwrap(rl_coalescer* c);

}  // namespace rlc
