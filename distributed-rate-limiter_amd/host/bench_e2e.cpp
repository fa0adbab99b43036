// bench_e2e.cpp -- BASELINE configs[4]: decision latency through the request
// coalescer at fixed offered QPS (open loop), adversarial Zipf s=1.5 over 1M
// keys (the top key is 38 % of the traffic), Token Bucket 100/min burst 20.
//
// G generator threads each emit a Poisson arrival process of rate QPS/G; every
// request due is submitted (all due requests of one thread in one submission)
// to the coalescer, which launches GPU batches through the engine.  A
// collector thread per generator waits for its submissions in order; a
// request's latency = completion time - its scheduled arrival time (so a late
// generator does not hide queueing: no coordinated omission).  Prints one
// JSON line with p50/p90/p99/p99.9 per QPS level.
#include <dirent.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <deque>
#include <mutex>
#include <condition_variable>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rl_engine.h"
#include "coalescer.hpp"

extern "C" int rl_engine_debug_q14_slow(rl_engine* e, uint64_t* out);   // diagnostic (rl_engine.hip)

namespace {

// runqueue wait (ns) of every thread of this process: /proc/self/task/*/schedstat
// field 2 (time spent runnable but not running)
std::vector<std::pair<long, uint64_t>> run_delays() {
    std::vector<std::pair<long, uint64_t>> out;
    DIR* d = opendir("/proc/self/task");
    if (!d) return out;
    while (dirent* e = readdir(d)) {
        if (e->d_name[0] == '.') continue;
        char path[128];
        snprintf(path, sizeof path, "/proc/self/task/%s/schedstat", e->d_name);
        FILE* f = fopen(path, "r");
        if (!f) continue;
        unsigned long long run = 0, wait = 0;
        if (fscanf(f, "%llu %llu", &run, &wait) == 2) out.push_back({atol(e->d_name), (uint64_t)wait});
        fclose(f);
    }
    closedir(d);
    return out;
}

size_t nb_cap(const std::string& slow) { return 4096 + slow.size(); }

constexpr int64_t NS = 1000000000LL;
constexpr int64_t T0_UNIX = 1760000000LL * NS;   // trace clock origin (as traces.py)

uint64_t splitmix(uint64_t x) {
    x += 0x9e3779b97f4a7c15ULL;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
    return x ^ (x >> 31);
}

// latency histogram: 0.1 us buckets to 1 ms, then 10 us buckets to 1 s
struct Hist {
    std::vector<uint64_t> fine = std::vector<uint64_t>(10000), coarse = std::vector<uint64_t>(100000);
    uint64_t count = 0, over = 0;
    void add(int64_t ns) {
        count++;
        if (ns < 0) ns = 0;
        if (ns < 1000000) fine[ns / 100]++;
        else if (ns < NS) coarse[ns / 10000]++;
        else over++;
    }
    void merge(const Hist& o) {
        for (size_t i = 0; i < fine.size(); i++) fine[i] += o.fine[i];
        for (size_t i = 0; i < coarse.size(); i++) coarse[i] += o.coarse[i];
        count += o.count;
        over += o.over;
    }
    double pct(double p) const {   // microseconds
        uint64_t want = (uint64_t)std::ceil(p / 100.0 * count), acc = 0;
        for (size_t i = 0; i < fine.size(); i++)
            if ((acc += fine[i]) >= want) return (i + 1) * 0.1;
        for (size_t i = 100; i < coarse.size(); i++)
            if ((acc += coarse[i]) >= want) return (i + 1) * 10.0;
        return 1e6;
    }
};

struct Pending {
    uint64_t ticket;
    std::vector<int64_t> arrival;   // scheduled arrival (steady ns) of each request
};

struct Args {
    std::vector<double> qps{1e5, 1e6, 1e7};
    double seconds = 2.0;
    uint32_t keys = 1000000;
    double zipf = 1.5;
    uint32_t max_batch = 1 << 18;
    int gens = 4;
    int device = 0;
    int64_t linger_ns = 0;
    int64_t limit = 20;          // Token Bucket 100/min burst 20 = {Limit 20, Window 12 s}
    double window_s = 12.0;
};

}  // namespace

int main(int argc, char** argv) {
    Args a;
    for (int i = 1; i + 1 < argc; i += 2) {
        std::string k = argv[i], v = argv[i + 1];
        if (k == "--qps") {
            a.qps.clear();
            size_t p = 0;
            while (p < v.size()) {
                size_t q = v.find(',', p);
                if (q == std::string::npos) q = v.size();
                a.qps.push_back(atof(v.substr(p, q - p).c_str()));
                p = q + 1;
            }
        } else if (k == "--seconds") a.seconds = atof(v.c_str());
        else if (k == "--keys") a.keys = (uint32_t)atol(v.c_str());
        else if (k == "--zipf") a.zipf = atof(v.c_str());
        else if (k == "--max-batch") a.max_batch = (uint32_t)atol(v.c_str());
        else if (k == "--gens") a.gens = atoi(v.c_str());
        else if (k == "--device") a.device = atoi(v.c_str());
        else if (k == "--linger-us") a.linger_ns = (int64_t)(atof(v.c_str()) * 1000);
        else if (k == "--limit") a.limit = atol(v.c_str());
        else if (k == "--window-s") a.window_s = atof(v.c_str());
        else { fprintf(stderr, "unknown option %s\n", k.c_str()); return 2; }
    }

    // key sample: Zipf(s) ranks -> ids through a seeded bijective mix
    std::vector<double> cdf(a.keys);
    double z = 0;
    for (uint32_t r = 0; r < a.keys; r++) cdf[r] = (z += std::pow(r + 1.0, -a.zipf));
    for (auto& x : cdf) x /= z;
    const size_t NSAMP = 1 << 22;
    std::vector<uint64_t> sample(NSAMP);
    std::mt19937_64 rng(5);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    for (auto& s : sample) {
        uint32_t r = (uint32_t)(std::lower_bound(cdf.begin(), cdf.end(), U(rng)) - cdf.begin());
        s = splitmix(r) >> 1;   // < RL_KEY_RESERVED
    }

    rl_opts o{};
    o.struct_size = sizeof o;
    o.device = a.device;
    o.profile = RL_PROFILE_REDIS7;
    o.tb_capacity = 1 << 21;
    o.win_capacity = 1024;
    o.max_batch = a.max_batch;
    o.flags = RL_OPT_PIPELINE;
    rl_engine* e = nullptr;
    if (rl_engine_create(&o, &e) != RL_OK) { fprintf(stderr, "engine create failed\n"); return 1; }
    uint32_t cfg = 0;
    if (rl_config_register(e, RL_ALG_TOKEN_BUCKET, a.limit, (int64_t)(a.window_s * NS), &cfg) != RL_OK) return 1;
    rl_coalescer_opts co{};
    co.struct_size = sizeof co;
    co.max_batch = a.max_batch;
    co.max_in_flight = 3;
    co.linger_ns = a.linger_ns;
    co.queue_cap = 1ull << 26;
    rl_coalescer* c = nullptr;
    if (rl_coalescer_create(e, &co, &c) != RL_OK) { fprintf(stderr, "coalescer create failed\n"); return 1; }

    std::string levels;
    int64_t trace_clock = 0;   // trace time continues across levels
    for (double qps : a.qps) {
        const int G = a.gens;
        const double rate = qps / G;   // per generator, per second
        rl_coalescer_stats s0{};
        s0.struct_size = sizeof s0;
        rl_coalescer_get_stats(c, &s0);
        std::vector<Hist> hist(G);
        // worst latency by arrival time, 100 ms buckets (where a tail comes from)
        const size_t NBK = (size_t)(a.seconds * 10) + 1;
        std::vector<std::vector<int64_t>> bmax(G, std::vector<int64_t>(NBK, 0));
        std::vector<uint64_t> sent(G, 0), dropped(G, 0);
        std::atomic<int64_t> last_done{0};
        const auto rd0 = run_delays();
        const int64_t start = rlc::steady_ns() + 20000000;   // 20 ms to spin up
        const int64_t stop = start + (int64_t)(a.seconds * NS);
        std::vector<std::thread> th;
        for (int g = 0; g < G; g++) {
            th.emplace_back([&, g] {
                std::mt19937_64 r(1000 + g + (uint64_t)qps);
                std::exponential_distribution<double> gap(rate / NS);   // ns
                std::deque<Pending> q;
                std::mutex qm;
                std::condition_variable qcv;
                bool fin = false;
                std::thread col([&] {
                    for (;;) {
                        Pending p;
                        {
                            std::unique_lock<std::mutex> lk(qm);
                            qcv.wait(lk, [&] { return fin || !q.empty(); });
                            if (q.empty()) return;
                            p = std::move(q.front());
                            q.pop_front();
                        }
                        int64_t done = 0;
                        rlc::unwrap(c)->Wait(p.ticket, -1, nullptr, nullptr, nullptr, nullptr, &done);
                        for (int64_t t : p.arrival) {
                            hist[g].add(done - t);
                            const size_t b = std::min<size_t>(NBK - 1, (size_t)std::max<int64_t>(0, (t - start) / 100000000));
                            bmax[g][b] = std::max<int64_t>(bmax[g][b], done - t);
                        }
                        int64_t prev = last_done.load();
                        while (done > prev && !last_done.compare_exchange_weak(prev, done)) {}
                    }
                });
                std::vector<uint64_t> key;
                std::vector<int64_t> ts, n;
                std::vector<uint32_t> cf;
                double next = (double)start + gap(r);
                size_t si = (size_t)(splitmix(g + 77) % NSAMP);
                while (rlc::steady_ns() < start) {}
                for (;;) {
                    int64_t now = rlc::steady_ns();
                    if (now >= stop) break;
                    if (next > now) continue;   // spin until the next arrival is due
                    key.clear(); ts.clear(); n.clear(); cf.clear();
                    std::vector<int64_t> arr;
                    while (next <= now && key.size() < 65536) {
                        arr.push_back((int64_t)next);
                        key.push_back(sample[si]);
                        si = (si + G) % NSAMP;
                        ts.push_back(T0_UNIX + trace_clock + ((int64_t)next - start));
                        n.push_back(1);
                        cf.push_back(cfg);
                        next += gap(r);
                    }
                    uint64_t t;
                    int rc = rl_coalescer_submit(c, key.size(), key.data(), ts.data(), n.data(), cf.data(), &t);
                    if (rc != RL_OK) { dropped[g] += key.size(); continue; }
                    sent[g] += key.size();
                    std::lock_guard<std::mutex> lk(qm);
                    q.push_back({t, std::move(arr)});
                    qcv.notify_one();
                }
                {
                    std::lock_guard<std::mutex> lk(qm);
                    fin = true;
                }
                qcv.notify_one();
                col.join();
            });
        }
        for (auto& t : th) t.join();
        trace_clock += (int64_t)(a.seconds * NS) + NS;
        // host scheduling: the largest runqueue wait any thread that lived
        // through the level accumulated during it (the coalescer's submitter
        // and completer among them)
        uint64_t max_rq = 0, sum_rq = 0;
        for (const auto& x : run_delays())
            for (const auto& y : rd0)
                if (x.first == y.first && x.second >= y.second) {
                    max_rq = std::max<uint64_t>(max_rq, x.second - y.second);
                    sum_rq += x.second - y.second;
                }
        Hist h;
        uint64_t tot = 0, drop = 0;
        for (int g = 0; g < G; g++) { h.merge(hist[g]); tot += sent[g]; drop += dropped[g]; }
        rl_coalescer_stats s1{};
        s1.struct_size = sizeof s1;
        rl_coalescer_get_stats(c, &s1);
        const double span = (double)(last_done.load() - start) / NS;
        const uint64_t nb = s1.batches - s0.batches;
        std::string tl;
        for (size_t b = 0; b < NBK; b++) {
            int64_t mx = 0;
            for (int g = 0; g < G; g++) mx = std::max(mx, bmax[g][b]);
            tl += (b ? ", " : "") + std::to_string(mx / 1000);
        }
        // stall attribution (RL_COALESCER_TRACE=<ring>): the batch whose oldest
        // request waited longest, split into queue (waiting for a launch slot),
        // stage-in (gather + H2D), enqueue (engine call), own device time (after
        // the previous batch's results were back) and in-order wait behind it
        std::string attr;
        {
            const std::vector<rlc::BatchTrace> tr = rlc::unwrap(c)->Trace();
            int64_t worst = -1;
            size_t wi = 0;
            double mx[5] = {0, 0, 0, 0, 0};
            std::string slow;   // [ms since start, stage-in us, enqueue us, own device us, m] of slow batches
            uint64_t traced = 0;
            for (size_t i = 1; i < tr.size(); i++) {
                const rlc::BatchTrace& t = tr[i];
                if (t.t_form < start) continue;
                traced++;
                const int64_t prev_done = tr[i - 1].t_done;
                const double q = (t.t_form - t.t_submit) / 1e3, si = (t.t_h2d - t.t_form) / 1e3,
                             en = (t.t_launched - t.t_h2d) / 1e3,
                             behind = (std::max(prev_done, t.t_launched) - t.t_launched) / 1e3,
                             own = (t.t_done - std::max(prev_done, t.t_launched)) / 1e3;
                const double v[5] = {q, si, en, behind, own};
                for (int k = 0; k < 5; k++) mx[k] = std::max(mx[k], v[k]);
                if (t.t_done - t.t_submit > worst) { worst = t.t_done - t.t_submit; wi = i; }
                if ((si > 1000 || en > 1000 || own > 1000) && slow.size() < 2000) {
                    char x[160];
                    snprintf(x, sizeof x, "%s[%.1f, %.0f, %.0f, %.0f, %llu]", slow.empty() ? "" : ", ",
                             (t.t_form - start) / 1e6, si, en, own, (unsigned long long)t.m);
                    slow += x;
                }
            }
            if (traced) {
                std::vector<char> abv(64 + nb_cap(slow));
                char* ab = abv.data();
                std::string nb;
                for (size_t i = wi >= 4 ? wi - 4 : 1; i <= wi + 1 && i < tr.size(); i++) {
                    const rlc::BatchTrace& t = tr[i];
                    const int64_t pd = tr[i - 1].t_done;
                    char x[256];
                    snprintf(x, sizeof x, "%s{\"m\": %llu, \"queue_us\": %.1f, \"stage_in_us\": %.1f, \"enqueue_us\": %.1f, "
                             "\"behind_prev_us\": %.1f, \"own_device_us\": %.1f}", nb.empty() ? "" : ", ",
                             (unsigned long long)t.m, (t.t_form - t.t_submit) / 1e3, (t.t_h2d - t.t_form) / 1e3,
                             (t.t_launched - t.t_h2d) / 1e3, (std::max(pd, t.t_launched) - t.t_launched) / 1e3,
                             (t.t_done - std::max(pd, t.t_launched)) / 1e3);
                    nb += x;
                }
                snprintf(ab, abv.size(),
                         ", \"trace\": {\"batches\": %llu, \"max_queue_us\": %.1f, \"max_stage_in_us\": %.1f, "
                         "\"max_enqueue_us\": %.1f, \"max_behind_prev_us\": %.1f, \"max_own_device_us\": %.1f, "
                         "\"worst_wait_us\": %.1f, \"worst_and_neighbours\": [%s], "
                         "\"slow_batches [ms, stage_in_us, enqueue_us, own_device_us, m]\": [%s]}",
                         (unsigned long long)traced, mx[0], mx[1], mx[2], mx[3], mx[4], worst / 1e3, nb.c_str(),
                         slow.c_str());
                attr = ab;
            }
        }
        std::vector<char> bufv(8192 + attr.size());
        char* buf = bufv.data();
        uint64_t slow_q14 = 0;
        (void)rl_engine_debug_q14_slow(e, &slow_q14);
        attr += ", \"q14_slow_calls_so_far\": " + std::to_string(slow_q14);
        attr += ", \"max_thread_runqueue_wait_us\": " + std::to_string(max_rq / 1000) +
                ", \"sum_thread_runqueue_wait_us\": " + std::to_string(sum_rq / 1000);
        snprintf(buf, bufv.size(),
                 "%s{\"offered_qps\": %.0f, \"achieved_decisions_per_s\": %.1f, \"requests\": %llu, \"dropped\": %llu, "
                 "\"p50_us\": %.1f, \"p90_us\": %.1f, \"p99_us\": %.1f, \"p999_us\": %.1f, \"batches\": %llu, "
                 "\"mean_batch\": %.1f, \"max_us_by_100ms\": [%s]%s}",
                 levels.empty() ? "" : ", ", qps, tot / span, (unsigned long long)tot, (unsigned long long)drop,
                 h.pct(50), h.pct(90), h.pct(99), h.pct(99.9), (unsigned long long)nb,
                 nb ? (double)(s1.decided - s0.decided) / nb : 0.0, tl.c_str(), attr.c_str());
        levels += buf;
        fprintf(stderr, "level %.0f qps done: %s\n", qps, buf);
    }
    rl_coalescer_destroy(c);
    int rc = rl_engine_sync(e);
    rl_engine_destroy(e);
    printf("{\"zipf\": %.2f, \"keys\": %u, \"gens\": %d, \"max_batch\": %u, \"linger_us\": %.1f, \"engine_status\": %d, "
           "\"levels\": [%s]}\n",
           a.zipf, a.keys, a.gens, a.max_batch, a.linger_ns / 1000.0, rc, levels.c_str());
    return rc == RL_OK ? 0 : 1;
}
