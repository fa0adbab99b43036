// rl_route.hip -- the routing kernels of include/rl_route.h: hash-sharded
// request batches across the GPUs of a node.
//
// All byte/integer work, HBM-bound, no MFMA, and no host round trip:
//   pack     owner hash, per-tile owner counts, one scan block per owner, a
//            stable scatter into fixed-capacity per-owner buckets of 32-byte
//            records (ranks from wave ballots, as rl_sort.h), so every split
//            of the all-to-alls is the same size and nothing is read back
//   merge    the received buckets in arrival order at one shared store: a
//            record arrives at the running max of its source's ts so far
//            (per-tile maxima, one scan block per source), ties go by (source
//            rank, source position); each source's bucket is already in
//            arrival order, so the order is a tree of ceil(log2 G) merge-path
//            merges (block splits by 64-ary wave searches, the tile merged in
//            LDS), the last level writing the decision order and each
//            request's store clock.  Sizes come from the received info rows,
//            in device memory; the store clock is a device word
//   unpack   32-byte result records back to the caller's order
// The engine reads the merged records itself (rl_decide_routed_device in
// rl_engine.hip) and writes result records at their receive index.
// Reference: the N app servers sharing one Redis of docs/ARCHITECTURE.md
// :142-164; the order one shared store applies a key's requests in.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "../../include/rl_route.h"
#include "rl_sort.h"
#include "rl_table.h"

using namespace rl;

namespace {

constexpr int RT_BLOCK = 256;
constexpr int RT_ITEMS = 4;                    // 1024-request tiles: ~1000 blocks per 1M batch
constexpr int RT_TILE = RT_BLOCK * RT_ITEMS;   // requests per pack tile
constexpr int MAX_WORLD = 64;

// router status bits (sticky, cleared by rl_router_sync)
constexpr uint32_t RS_OVERFLOW = 1u;           // a request was dropped: its owner's bucket was full

__device__ inline uint32_t owner_of(uint64_t k, uint32_t world) { return (uint32_t)(mix64(k) >> 32) % world; }

// lanes of this wave holding the same owner id as this lane (ballots over the
// id's bits; world <= 64, so at most 6), restricted to `valid`
__device__ inline uint64_t owner_peers(uint32_t own, uint32_t world, bool valid) {
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 6; b++) {
        if ((1u << b) >= world) break;   // wave-uniform
        const uint32_t bit = (own >> b) & 1u;
        const uint64_t bb = __ballot(bit);
        peers &= bit ? bb : ~bb;
    }
    return peers;
}

__global__ __launch_bounds__(RT_BLOCK) void k_route_owner(uint32_t m, const uint64_t* __restrict__ key,
                                                          uint32_t world, uint32_t* __restrict__ owner) {
    for (uint32_t i = blockIdx.x * RT_BLOCK + threadIdx.x; i < m; i += gridDim.x * RT_BLOCK)
        owner[i] = owner_of(key[i], world);
}

__device__ inline unsigned long long bias(int64_t t) { return (unsigned long long)t ^ 0x8000000000000000ull; }
__device__ inline int64_t unbias(unsigned long long u) { return (int64_t)(u ^ 0x8000000000000000ull); }

// summary of a batch (pack): earliest / latest ts (biased), whether ts ever
// decreases (a source in time order needs no running max at its owners)
struct PackSum {
    unsigned long long lo, hi;
    uint32_t unsorted;
};


// per-tile owner counts: tile_cnt[tile * world + o]; the tile's summary in
// tile_sum[tile] (no global atomics: k_route_scan reduces the tiles)
__global__ __launch_bounds__(RT_BLOCK) void k_route_hist(uint32_t m, const uint64_t* __restrict__ key,
                                                         const int64_t* __restrict__ ts, uint32_t world,
                                                         uint32_t* __restrict__ tile_cnt, PackSum* tile_sum) {
    __shared__ uint32_t s_cnt[MAX_WORLD];
    __shared__ unsigned long long s_lo[RT_BLOCK / 64], s_hi[RT_BLOCK / 64];
    __shared__ uint32_t s_uns;
    if (threadIdx.x < MAX_WORLD) s_cnt[threadIdx.x] = 0;
    if (threadIdx.x == 0) s_uns = 0;
    __syncthreads();
    const uint32_t base = blockIdx.x * RT_TILE;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t lt = (1ull << lane) - 1ull;
    unsigned long long lo = ~0ull, hi = 0;
    uint32_t uns = 0;
#pragma unroll
    for (int j = 0; j < RT_ITEMS; j++) {
        const uint32_t i = base + j * RT_BLOCK + threadIdx.x;
        const bool ok = i < m;
        const uint32_t own = ok ? owner_of(key[i], world) : 0u;
        const int64_t t = ok ? ts[i] : 0;
        // a wave's 64 requests are consecutive: the predecessor's ts is the
        // lane below (lane 0 loads it)
        int64_t tp = __shfl_up(t, 1);
        if (lane == 0) tp = (ok && i > 0) ? ts[i - 1] : t;
        if (ok && i > 0 && tp > t) uns = 1;
        // one LDS add per owner per wave (not per request: at small world
        // every request of a tile would hit one counter)
        const uint64_t peers = owner_peers(own, world, ok);
        if (ok && (peers & lt) == 0) atomicAdd(&s_cnt[own], (uint32_t)__popcll(peers));
        if (ok) {
            const unsigned long long b = bias(t);
            lo = b < lo ? b : lo;
            hi = b > hi ? b : hi;
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long l2 = __shfl_xor(lo, off), h2 = __shfl_xor(hi, off);
        lo = l2 < lo ? l2 : lo;
        hi = h2 > hi ? h2 : hi;
    }
    if ((threadIdx.x & 63) == 0) {
        s_lo[threadIdx.x >> 6] = lo;
        s_hi[threadIdx.x >> 6] = hi;
    }
    if (uns) s_uns = 1;   // benign race: every writer stores 1
    __syncthreads();
    if (threadIdx.x == 0) {
        PackSum t{~0ull, 0ull, s_uns};
        for (int w = 0; w < RT_BLOCK / 64; w++) {
            t.lo = s_lo[w] < t.lo ? s_lo[w] : t.lo;
            t.hi = s_hi[w] > t.hi ? s_hi[w] : t.hi;
        }
        tile_sum[blockIdx.x] = t;
    }
    if (threadIdx.x < world) tile_cnt[(size_t)blockIdx.x * world + threadIdx.x] = s_cnt[threadIdx.x];
}


// block o: owner o's bucket offset per tile (an exclusive prefix over the
// tiles) into tile_off, and owner o's info row {sent (<= cap), earliest ts,
// latest ts, dropped}
__global__ __launch_bounds__(RT_BLOCK) void k_route_scan(uint32_t tiles, uint32_t world, uint32_t cap,
                                                         const uint32_t* __restrict__ tile_cnt,
                                                         uint32_t* __restrict__ tile_off,
                                                         const PackSum* __restrict__ tile_sum,
                                                         int64_t* __restrict__ info) {
    __shared__ uint32_t s_tmp[RT_BLOCK / 64];
    __shared__ unsigned long long s_lo[RT_BLOCK / 64], s_hi[RT_BLOCK / 64];
    __shared__ uint32_t s_uns;
    const uint32_t o = blockIdx.x, tid = threadIdx.x;
    if (tid == 0) s_uns = 0;
    __syncthreads();
    // the batch summary from the tiles' summaries
    unsigned long long lo = ~0ull, hi = 0;
    uint32_t uns = 0;
    for (uint32_t t = tid; t < tiles; t += RT_BLOCK) {
        const PackSum ps = tile_sum[t];
        lo = ps.lo < lo ? ps.lo : lo;
        hi = ps.hi > hi ? ps.hi : hi;
        uns |= ps.unsorted;
    }
    if (uns) s_uns = 1;
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long l2 = __shfl_xor(lo, off), h2 = __shfl_xor(hi, off);
        lo = l2 < lo ? l2 : lo;
        hi = h2 > hi ? h2 : hi;
    }
    if ((tid & 63) == 0) {
        s_lo[tid >> 6] = lo;
        s_hi[tid >> 6] = hi;
    }
    uint32_t run = 0;
    for (uint32_t t0 = 0; t0 < tiles; t0 += RT_BLOCK) {
        const uint32_t t = t0 + tid;
        const uint32_t c = t < tiles ? tile_cnt[(size_t)t * world + o] : 0u;
        uint32_t inc = wave_incl_scan(c, tid & 63);
        __syncthreads();
        if ((tid & 63) == 63) s_tmp[tid >> 6] = inc;
        __syncthreads();
        uint32_t pre = 0, tot = 0;
        for (int w = 0; w < RT_BLOCK / 64; w++) {
            if (w < (int)(tid >> 6)) pre += s_tmp[w];
            tot += s_tmp[w];
        }
        if (t < tiles) tile_off[(size_t)t * world + o] = run + pre + inc - c;
        run += tot;
    }
    if (tid == 0) {
        for (int w = 0; w < RT_BLOCK / 64; w++) {
            lo = s_lo[w] < lo ? s_lo[w] : lo;
            hi = s_hi[w] > hi ? s_hi[w] : hi;
        }
        int64_t* row = info + (size_t)RL_ROUTE_INFO * o;
        row[0] = run < cap ? run : cap;
        row[1] = tiles ? unbias(lo) : INT64_MAX;
        row[2] = tiles ? unbias(hi) : INT64_MIN;
        // dropped requests, and bit 0: the batch's ts decrease somewhere
        row[3] = (int64_t)(run > cap ? run - cap : 0) * 2 + (s_uns ? 1 : 0);
    }
}

// stable scatter of the requests into their owners' buckets; past a bucket's
// capacity a request is dropped (slot UINT32_MAX, sticky RS_OVERFLOW)
__global__ __launch_bounds__(RT_BLOCK) void k_route_scatter(uint32_t m, const uint64_t* __restrict__ key,
                                                            const int64_t* __restrict__ ts,
                                                            const int64_t* __restrict__ n,
                                                            const uint32_t* __restrict__ cfg, uint32_t world,
                                                            uint32_t cap, const uint32_t* __restrict__ tile_off,
                                                            rl_route_rec* __restrict__ send,
                                                            uint32_t* __restrict__ slot, uint32_t* status) {
    constexpr int W = RT_BLOCK / 64;
    __shared__ uint32_t s_wcnt[W][MAX_WORLD];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int k = tid; k < W * MAX_WORLD; k += RT_BLOCK) (&s_wcnt[0][0])[k] = 0;
    __syncthreads();
    // wave w takes the tile's requests [w * 64 * RT_ITEMS, (w + 1) * 64 * RT_ITEMS) in order
    const uint32_t base = blockIdx.x * RT_TILE + wave * (64 * RT_ITEMS);
    uint32_t own[RT_ITEMS], rank[RT_ITEMS];
    const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll
    for (int j = 0; j < RT_ITEMS; j++) {
        const uint32_t i = base + j * 64 + lane;
        const bool ok = i < m;
        own[j] = ok ? owner_of(key[i], world) : 0u;
        const uint64_t peers = owner_peers(own[j], world, ok);
        if (ok) {
            const uint32_t below = __popcll(peers & lt);
            const uint32_t cur = s_wcnt[wave][own[j]];
            rank[j] = cur + below;
            if (below == 0) s_wcnt[wave][own[j]] = cur + (uint32_t)__popcll(peers);
        }
    }
    __syncthreads();
    // per owner: exclusive prefix over the waves, plus the tile's offset
    if (tid < (int)world) {
        uint32_t run = tile_off[(size_t)blockIdx.x * world + tid];
        for (int w = 0; w < W; w++) {
            const uint32_t c = s_wcnt[w][tid];
            s_wcnt[w][tid] = run;
            run += c;
        }
    }
    __syncthreads();
    bool over = false;
#pragma unroll
    for (int j = 0; j < RT_ITEMS; j++) {
        const uint32_t i = base + j * 64 + lane;
        if (i >= m) continue;
        const uint32_t p = s_wcnt[wave][own[j]] + rank[j];
        if (p >= cap) {
            slot[i] = 0xffffffffu;
            over = true;
            continue;
        }
        rl_route_rec r;
        r.key = key[i];
        r.ts = ts[i];
        r.n = n[i];
        r.cfg = cfg[i];
        r.pos = i;
        const uint32_t at = own[j] * cap + p;
        send[at] = r;
        slot[i] = at;
    }
    if (__ballot(over) && lane == 0) atomicOr(status, RS_OVERFLOW);
}

// ---- the merge, planned on the device ---------------------------------------
constexpr int MT_ITEMS = 4;                       // consecutive records per thread (arrival scans)
constexpr uint32_t MT_TILE = RT_BLOCK * MT_ITEMS;
constexpr int MP_ITEMS = 8;                       // outputs per thread of a merge-path tile
constexpr uint32_t MP_TILE = RT_BLOCK * MP_ITEMS;
constexpr uint32_t CAP_ALIGN = MP_TILE;           // bucket capacities are multiples of this
static_assert(CAP_ALIGN % MT_TILE == 0, "tiles never straddle buckets");
constexpr unsigned long long TS_BIAS = 1ull << 63;   // int64 order as uint64 order

// the merge's control words (one step at a time: merges run in step order)
struct MergeCtl {
    int64_t clock_prev;            // the store clock of the earlier steps (ms)
    uint32_t len[MAX_WORLD];       // records received from each source (<= cap)
};

__device__ inline uint32_t recv_count(const int64_t* __restrict__ info, uint32_t s, uint32_t cap) {
    const int64_t c = info[(size_t)RL_ROUTE_INFO * s];
    return c <= 0 ? 0u : (c >= (int64_t)cap ? cap : (uint32_t)c);
}
// the source's batch never goes back in time: arrival = ts, no running max
__device__ inline bool recv_sorted(const int64_t* __restrict__ info, uint32_t s) {
    return (info[(size_t)RL_ROUTE_INFO * s + 3] & 1) == 0;
}

// per tile of MT_TILE received records: the max biased ts (scan inputs).
// Tile t is source t / tps's tile t % tps.
__global__ __launch_bounds__(RT_BLOCK) void k_bm_tmax(const rl_route_rec* __restrict__ rec,
                                                      const int64_t* __restrict__ info, uint32_t cap, uint32_t tps,
                                                      unsigned long long* __restrict__ tmax) {
    __shared__ unsigned long long s_w[RT_BLOCK / 64];
    const uint32_t s = blockIdx.x / tps, u = blockIdx.x % tps;
    const uint32_t c = recv_count(info, s, cap);
    if (recv_sorted(info, s)) return;   // block-uniform: no scan inputs needed
    unsigned long long mx = 0;
    if (u * MT_TILE < c) {
#pragma unroll
        for (int q = 0; q < MT_ITEMS; q++) {
            const uint32_t i = u * MT_TILE + threadIdx.x * MT_ITEMS + q;
            if (i < c) {
                const unsigned long long b = (unsigned long long)rec[(size_t)s * cap + i].ts ^ TS_BIAS;
                mx = b > mx ? b : mx;
            }
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(mx, off);
        mx = o > mx ? o : mx;
    }
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < RT_BLOCK / 64; w++) mx = s_w[w] > mx ? s_w[w] : mx;
        tmax[blockIdx.x] = mx;
    }
}

// block s: exclusive running max over source s's tiles (in place).  Block 0
// also takes the step's sizes and advances the store clock: every owner sees
// the same info rows, so every owner keeps the same clock
__global__ __launch_bounds__(1024) void k_bm_tscan(const int64_t* __restrict__ info, uint32_t world, uint32_t cap,
                                                   uint32_t tps, unsigned long long* tmax, int64_t* clock,
                                                   MergeCtl* ctl, uint32_t* count, uint32_t* order, int64_t* sms) {
    __shared__ unsigned long long s_w[16];
    __shared__ unsigned long long s_carry;
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t s = blockIdx.x;
    const uint32_t tiles = recv_sorted(info, s) ? 0u : (recv_count(info, s, cap) + MT_TILE - 1) / MT_TILE;
    unsigned long long* t_s = tmax + (size_t)s * tps;
    if (tid == 0) s_carry = 0;
    __syncthreads();
    for (uint32_t t0 = 0; t0 < tiles; t0 += 1024) {
        const uint32_t t = t0 + tid;
        const unsigned long long v = t < tiles ? t_s[t] : 0ull;
        unsigned long long inc = v;
        for (int o = 1; o < 64; o <<= 1) {
            const unsigned long long u = __shfl_up(inc, o, 64);
            if (lane >= (uint32_t)o) inc = u > inc ? u : inc;
        }
        if (lane == 63) s_w[w] = inc;
        __syncthreads();
        unsigned long long pre = s_carry;
        for (uint32_t k = 0; k < w; k++) pre = s_w[k] > pre ? s_w[k] : pre;
        unsigned long long ex = __shfl_up(inc, 1, 64);
        ex = lane ? (ex > pre ? ex : pre) : pre;
        __syncthreads();
        if (t < tiles) t_s[t] = ex;   // exclusive: the max of every earlier record of the source
        if (tid == 1023) s_carry = inc > pre ? inc : pre;
        __syncthreads();
    }
    if (s == 0 && tid == 0) {
        const int64_t c0 = *clock;
        int64_t c1 = c0;
        uint32_t tot = 0;
        for (uint32_t q = 0; q < world; q++) {
            const int64_t latest = info[(size_t)RL_ROUTE_INFO * q + 2];
            if (latest != INT64_MIN) {   // after this step: clock = max(clock, floor(latest ts / 1e6))
                const int64_t ms = floor_div(latest, 1000000LL);
                c1 = ms > c1 ? ms : c1;
            }
            const uint32_t c = recv_count(info, q, cap);
            ctl->len[q] = c;
            tot += c;
        }
        ctl->clock_prev = c0;
        *clock = c1;
        *count = tot;
        // one source in time order: the received order is the decision order
        // and each request's clock follows from its own ts (RL_ORDER_IDENTITY)
        if (world == 1 && recv_sorted(info, 0)) {
            order[0] = RL_ORDER_IDENTITY;
            sms[0] = c0;
        }
    }
}

// every received record's arrival (biased): the running max of its source's
// ts so far.  One source (world 1): the received order is the decision order,
// so the order and store clocks are written here and nothing else runs (and
// nothing at all for one source in time order: RL_ORDER_IDENTITY).
__global__ __launch_bounds__(RT_BLOCK) void k_bm_keys(const rl_route_rec* __restrict__ rec,
                                                      const int64_t* __restrict__ info, uint32_t world, uint32_t cap,
                                                      uint32_t tps, const unsigned long long* __restrict__ tpre,
                                                      const MergeCtl* __restrict__ ctl,
                                                      unsigned long long* __restrict__ akey,
                                                      uint32_t* __restrict__ order, int64_t* __restrict__ sms) {
    __shared__ unsigned long long s_w[RT_BLOCK / 64];
    const uint32_t s = blockIdx.x / tps, u = blockIdx.x % tps;
    const uint32_t c = recv_count(info, s, cap);
    if (u * MT_TILE >= c) return;   // block-uniform
    if (world == 1 && recv_sorted(info, 0)) return;   // RL_ORDER_IDENTITY (k_bm_tscan)
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t i0 = u * MT_TILE + threadIdx.x * MT_ITEMS;
    const bool sorted = recv_sorted(info, s);    // block-uniform
    unsigned long long a[MT_ITEMS];
    unsigned long long run = 0;
#pragma unroll
    for (int q = 0; q < MT_ITEMS; q++) {
        const uint32_t i = i0 + q;
        a[q] = i < c ? (unsigned long long)rec[(size_t)s * cap + i].ts ^ TS_BIAS : 0ull;
        run = a[q] > run ? a[q] : run;
        if (!sorted) a[q] = run;                 // inclusive within the thread
    }
    unsigned long long ex = 0;
    if (!sorted) {
        unsigned long long inc = run;
        for (int o = 1; o < 64; o <<= 1) {
            const unsigned long long v = __shfl_up(inc, o, 64);
            if (lane >= (uint32_t)o) inc = v > inc ? v : inc;
        }
        if (lane == 63) s_w[w] = inc;
        __syncthreads();
        unsigned long long pre = tpre[blockIdx.x];
        for (uint32_t k = 0; k < w; k++) pre = s_w[k] > pre ? s_w[k] : pre;
        ex = __shfl_up(inc, 1, 64);
        ex = lane ? (ex > pre ? ex : pre) : pre;
    }
    const int64_t c0 = ctl->clock_prev;
#pragma unroll
    for (int q = 0; q < MT_ITEMS; q++) {
        const uint32_t i = i0 + q;
        if (i >= c) continue;
        const unsigned long long arrive = a[q] > ex ? a[q] : ex;
        if (world == 1) {
            const int64_t ms = floor_div((int64_t)(arrive ^ TS_BIAS), 1000000LL);
            order[i] = i;
            sms[i] = ms > c0 ? ms : c0;
        } else {
            akey[(size_t)s * cap + i] = arrive;
        }
    }
}

// merge path: the number of list-A elements among the first d outputs of
// merging A (la) and B (lb), ties to A (the lower source ranks) -- the first
// a in [max(0, d - lb), min(d, la)] with NOT A[a] <= B[d - a - 1].  One wave,
// 64-ary: each round every lane tests one candidate.
__device__ inline uint32_t wave_split(const unsigned long long* __restrict__ A, uint32_t la,
                                      const unsigned long long* __restrict__ B, uint32_t lb, uint32_t d) {
    const uint32_t lane = threadIdx.x & 63;
    uint32_t lo = d > lb ? d - lb : 0u, hi = d < la ? d : la;
    while (lo < hi) {
        const uint32_t n = hi - lo;
        const uint32_t step = (n + 63) / 64;
        const uint32_t a = lo + lane * step;
        const bool ok = lane * step < n && A[a] <= B[d - a - 1];
        const uint32_t c = (uint32_t)__popcll(__ballot(ok));   // the true candidates are a prefix
        if (c == 0) break;                                     // the answer is lo
        const uint32_t nlo = lo + (c - 1) * step + 1;
        const uint32_t nhi = lo + c * step;
        lo = nlo;
        hi = nhi < hi ? nhi : hi;
    }
    return lo;
}
__device__ inline uint32_t lds_split(const unsigned long long* A, uint32_t la, const unsigned long long* B,
                                     uint32_t lb, uint32_t d) {
    uint32_t lo = d > lb ? d - lb : 0u, hi = d < la ? d : la;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (A[mid] <= B[d - mid - 1]) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// One level of the merge tree: level-l lists are the sources [k 2^l, (k+1) 2^l),
// stored at k * 2^l * cap; lists 2k and 2k+1 merge into level-(l+1) list k.
// Block b covers output positions [b MP_TILE, (b+1) MP_TILE) of the level's
// world * cap.  Level 0 lists are the sources' buckets (values implicit: the
// receive index).  The last level writes the decision order and store clocks.
template <bool LAST>
__global__ __launch_bounds__(RT_BLOCK) void k_bm_merge(uint32_t level, uint32_t world, uint32_t cap,
                                                       const MergeCtl* __restrict__ ctl,
                                                       const unsigned long long* __restrict__ kin,
                                                       const uint32_t* __restrict__ vin,
                                                       unsigned long long* __restrict__ kout,
                                                       uint32_t* __restrict__ vout, uint32_t* __restrict__ order,
                                                       int64_t* __restrict__ sms) {
    __shared__ unsigned long long s_k[MP_TILE];
    __shared__ uint32_t s_v[MP_TILE];
    __shared__ uint32_t s_split[2];
    const uint64_t span_in = (uint64_t)cap << level, span_out = span_in << 1;
    const uint64_t e0 = (uint64_t)blockIdx.x * MP_TILE;
    const uint32_t k = (uint32_t)(e0 / span_out);
    const uint32_t d0 = (uint32_t)(e0 - k * span_out);
    const uint32_t sa = (2u * k) << level, sb = (2u * k + 1u) << level, se = (2u * k + 2u) << level;
    uint32_t la = 0, lb = 0;
    for (uint32_t q = sa; q < world && q < se; q++) (q < sb ? la : lb) += ctl->len[q];
    if (d0 >= la + lb) return;   // block-uniform
    const uint32_t d1 = d0 + MP_TILE < la + lb ? d0 + MP_TILE : la + lb;
    const uint64_t aoff = (uint64_t)k * span_out, boff = aoff + span_in;
    const unsigned long long* A = kin + aoff;
    const unsigned long long* B = kin + boff;
    const uint32_t wave = threadIdx.x >> 6;
    if (wave < 2) {
        const uint32_t a = wave_split(A, la, B, lb, wave ? d1 : d0);
        if ((threadIdx.x & 63) == 0) s_split[wave] = a;
    }
    __syncthreads();
    const uint32_t a0 = s_split[0], a1 = s_split[1];
    const uint32_t b0 = d0 - a0, b1 = d1 - a1;
    const uint32_t na = a1 - a0, nb = b1 - b0;
    for (uint32_t i = threadIdx.x; i < na + nb; i += RT_BLOCK) {
        const bool fa = i < na;
        const uint64_t at = fa ? aoff + a0 + i : boff + b0 + (i - na);
        s_k[i] = kin[at];
        s_v[i] = vin ? vin[at] : (uint32_t)at;   // level 0: the receive index
    }
    __syncthreads();
    const uint32_t n = d1 - d0;
    const uint32_t dl = threadIdx.x * MP_ITEMS;
    if (dl >= n) return;
    const unsigned long long* As = s_k;
    const unsigned long long* Bs = s_k + na;
    uint32_t i = lds_split(As, na, Bs, nb, dl), j = dl - i;
    const int64_t c0 = LAST ? ctl->clock_prev : 0;
#pragma unroll
    for (int q = 0; q < MP_ITEMS; q++) {
        const uint32_t dd = dl + q;
        if (dd >= n) break;
        const bool takeA = j >= nb || (i < na && As[i] <= Bs[j]);
        const unsigned long long key = takeA ? As[i] : Bs[j];
        const uint32_t v = takeA ? s_v[i] : s_v[na + j];
        if (takeA) i++;
        else j++;
        const uint64_t out = aoff + d0 + dd;
        if (LAST) {
            const int64_t ms = floor_div((int64_t)(key ^ TS_BIAS), 1000000LL);
            order[out] = v;
            sms[out] = ms > c0 ? ms : c0;
        } else {
            kout[out] = key;
            vout[out] = v;
        }
    }
}

// Results into the caller's order, one request per thread.  In a routed step
// its kernel-trace time (64-67 us per 1M requests) is contention with the
// replay and the next batch's grouping running beside it: alone it takes
// 10 us (5.9 TB/s of its 61 bytes per request; profiles/r5m_route_unpack.txt).
__device__ inline void unpack_one(uint32_t s, const rl_route_res* __restrict__ back, uint32_t& d, int64_t& rm,
                                  int64_t& rt, int64_t& rs) {
    if (s == 0xffffffffu) {   // dropped at the sender: never executed
        d = RL_DROPPED;
        rm = rt = rs = 0;
        return;
    }
    const rl_route_res r = back[s];
    d = (uint32_t)(uint8_t)r.decision;
    rm = r.remaining;
    rt = r.retry_after_ns;
    rs = r.reset_at_ns;
}
__global__ __launch_bounds__(RT_BLOCK) void k_route_unpack(uint32_t m, const uint32_t* __restrict__ slot,
                                                           const rl_route_res* __restrict__ back,
                                                           uint8_t* __restrict__ dec, int64_t* __restrict__ rem,
                                                           int64_t* __restrict__ retry,
                                                           int64_t* __restrict__ reset) {
    for (uint32_t i = blockIdx.x * RT_BLOCK + threadIdx.x; i < m; i += gridDim.x * RT_BLOCK) {
        uint32_t d;
        int64_t rm, rt, rs;
        unpack_one(slot[i], back, d, rm, rt, rs);
        dec[i] = (uint8_t)d;
        rem[i] = rm;
        retry[i] = rt;
        reset[i] = rs;
    }
}

int grid_for(size_t m) { return (int)std::min<size_t>((m + RT_BLOCK - 1) / RT_BLOCK, 2048); }

}  // namespace

struct rl_router {
    int device = 0;
    uint32_t world = 1, max_batch = 0, cap = 0;
    uint32_t* tile_cnt = nullptr;    // pack: [tiles][world]
    uint32_t* tile_off = nullptr;    // pack: [tiles][world] bucket offsets
    PackSum* psum = nullptr;         // pack: per-tile summaries [tiles]
    unsigned long long* tmax = nullptr;           // merge: per-tile running-max scan [world * cap / MT_TILE]
    unsigned long long *ak0 = nullptr, *ak1 = nullptr;   // merge: arrival keys (ping-pong) [world * cap]
    uint32_t *iv0 = nullptr, *iv1 = nullptr;      // merge: receive indices (ping-pong) [world * cap]
    MergeCtl* ctl = nullptr;
    int64_t* d_clock = nullptr;      // the store clock of the next step (ms)
    uint32_t* d_status = nullptr;    // sticky router status (RS_*)
};

extern "C" int rl_router_create(int32_t device, int32_t world, uint32_t max_batch, uint32_t cap, rl_router** out) {
    if (!out || world < 1 || world > MAX_WORLD || max_batch == 0 || cap == 0 || max_batch > (1u << 30) ||
        (uint64_t)cap * (uint64_t)world > (1u << 30))
        return RL_EINVAL;
    *out = nullptr;
    if (hipSetDevice(device) != hipSuccess) return RL_EDEVICE;
    rl_router* r = new rl_router();
    r->device = device;
    r->world = (uint32_t)world;
    r->max_batch = max_batch;
    r->cap = (cap + CAP_ALIGN - 1) / CAP_ALIGN * CAP_ALIGN;
    const size_t ptiles = (max_batch + RT_TILE - 1) / RT_TILE;
    const size_t tot = (size_t)r->cap * world;
    bool ok = hipMalloc(&r->tile_cnt, 4 * ptiles * world) == hipSuccess;
    ok = ok && hipMalloc(&r->tile_off, 4 * ptiles * world) == hipSuccess;
    ok = ok && hipMalloc(&r->psum, sizeof(PackSum) * ptiles) == hipSuccess;
    ok = ok && hipMalloc(&r->tmax, 8 * (tot / MT_TILE)) == hipSuccess;
    if (world > 1) {
        ok = ok && hipMalloc(&r->ak0, 8 * tot) == hipSuccess && hipMalloc(&r->ak1, 8 * tot) == hipSuccess;
        ok = ok && hipMalloc(&r->iv0, 4 * tot) == hipSuccess && hipMalloc(&r->iv1, 4 * tot) == hipSuccess;
    }
    ok = ok && hipMalloc(&r->ctl, sizeof(MergeCtl)) == hipSuccess;
    ok = ok && hipMalloc(&r->d_clock, 8) == hipSuccess;
    ok = ok && hipMalloc(&r->d_status, 4) == hipSuccess && hipMemset(r->d_status, 0, 4) == hipSuccess;
    const int64_t c0 = INT64_MIN;
    ok = ok && hipMemcpy(r->d_clock, &c0, 8, hipMemcpyHostToDevice) == hipSuccess;
    if (!ok) {
        rl_router_destroy(r);
        return RL_ENOMEM;
    }
    *out = r;
    return RL_OK;
}

extern "C" int rl_router_destroy(rl_router* r) {
    if (!r) return RL_EINVAL;
    (void)hipSetDevice(r->device);
    for (void* p : {(void*)r->tile_cnt, (void*)r->tile_off, (void*)r->psum, (void*)r->tmax, (void*)r->ak0,
                    (void*)r->ak1, (void*)r->iv0, (void*)r->iv1, (void*)r->ctl, (void*)r->d_clock,
                    (void*)r->d_status})
        (void)hipFree(p);
    delete r;
    return RL_OK;
}

extern "C" uint32_t rl_router_capacity(const rl_router* r) { return r ? r->cap : 0u; }

extern "C" int rl_router_sync(rl_router* r, void* stream) {
    if (!r) return RL_EINVAL;
    (void)hipSetDevice(r->device);
    if (hipStreamSynchronize((hipStream_t)stream) != hipSuccess) return RL_EDEVICE;
    uint32_t s = 0;
    if (hipMemcpy(&s, r->d_status, 4, hipMemcpyDeviceToHost) != hipSuccess) return RL_EDEVICE;
    if (hipMemset(r->d_status, 0, 4) != hipSuccess) return RL_EDEVICE;
    return (s & RS_OVERFLOW) ? RL_EOVERFLOW : RL_OK;
}

extern "C" int rl_stream_create_dedicated(int32_t device, void** out) {
    if (!out) return RL_EINVAL;
    *out = nullptr;
    if (hipSetDevice(device) != hipSuccess) return RL_EDEVICE;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return RL_EDEVICE;
    const int ncu = prop.multiProcessorCount;
    std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
    for (int c = 0; c < ncu; c++) mask[c / 32] |= 1u << (c % 32);
    hipStream_t st = nullptr;
    if (hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data()) != hipSuccess) return RL_EDEVICE;
    *out = st;
    return RL_OK;
}

extern "C" int rl_stream_destroy(void* stream) {
    if (!stream) return RL_EINVAL;
    return hipStreamDestroy((hipStream_t)stream) == hipSuccess ? RL_OK : RL_EDEVICE;
}

extern "C" int rl_route_owner(rl_router* r, size_t m, const uint64_t* key, uint32_t* owner, void* stream) {
    if (!r || (m && (!key || !owner)) || m > r->max_batch) return RL_EINVAL;
    if (!m) return RL_OK;
    (void)hipSetDevice(r->device);
    k_route_owner<<<grid_for(m), RT_BLOCK, 0, (hipStream_t)stream>>>((uint32_t)m, key, r->world, owner);
    return hipGetLastError() == hipSuccess ? RL_OK : RL_EDEVICE;
}

extern "C" int rl_route_pack(rl_router* r, size_t m, const uint64_t* key, const int64_t* ts, const int64_t* n,
                             const uint32_t* cfg, rl_route_rec* send, int64_t* send_info, uint32_t* slot,
                             void* stream) {
    if (!r || !send_info || m > r->max_batch || (m && (!key || !ts || !n || !cfg || !send || !slot)))
        return RL_EINVAL;
    (void)hipSetDevice(r->device);
    hipStream_t s = (hipStream_t)stream;
    const uint32_t tiles = (uint32_t)((m + RT_TILE - 1) / RT_TILE);
    if (m) k_route_hist<<<tiles, RT_BLOCK, 0, s>>>((uint32_t)m, key, ts, r->world, r->tile_cnt, r->psum);
    k_route_scan<<<r->world, RT_BLOCK, 0, s>>>(tiles, r->world, r->cap, r->tile_cnt, r->tile_off, r->psum, send_info);
    if (m)
        k_route_scatter<<<tiles, RT_BLOCK, 0, s>>>((uint32_t)m, key, ts, n, cfg, r->world, r->cap, r->tile_off, send,
                                                   slot, r->d_status);
    return hipGetLastError() == hipSuccess ? RL_OK : RL_EDEVICE;
}

extern "C" int rl_route_merge(rl_router* r, const rl_route_rec* recv, const int64_t* recv_info, uint32_t* order,
                              int64_t* server_ms, uint32_t* count, void* stream) {
    if (!r || !recv || !recv_info || !order || !server_ms || !count) return RL_EINVAL;
    (void)hipSetDevice(r->device);
    hipStream_t s = (hipStream_t)stream;
    const uint32_t G = r->world, cap = r->cap;
    const uint32_t tps = cap / MT_TILE;
    k_bm_tmax<<<G * tps, RT_BLOCK, 0, s>>>(recv, recv_info, cap, tps, r->tmax);
    k_bm_tscan<<<G, 1024, 0, s>>>(recv_info, G, cap, tps, r->tmax, r->d_clock, r->ctl, count, order, server_ms);
    k_bm_keys<<<G * tps, RT_BLOCK, 0, s>>>(recv, recv_info, G, cap, tps, r->tmax, r->ctl, r->ak0, order, server_ms);
    // the merge tree: ceil(log2 G) levels, ping-pong between (ak0, iv0) and (ak1, iv1)
    uint32_t levels = 0;
    while ((1u << levels) < G) levels++;
    const uint32_t blocks = G * (cap / MP_TILE);
    unsigned long long *kin = r->ak0, *kout = r->ak1;
    uint32_t *vin = nullptr, *vout = r->iv1;
    for (uint32_t l = 0; l < levels; l++) {
        if (l + 1 == levels)
            k_bm_merge<true><<<blocks, RT_BLOCK, 0, s>>>(l, G, cap, r->ctl, kin, vin, nullptr, nullptr, order,
                                                         server_ms);
        else
            k_bm_merge<false><<<blocks, RT_BLOCK, 0, s>>>(l, G, cap, r->ctl, kin, vin, kout, vout, nullptr, nullptr);
        std::swap(kin, kout);
        vin = vout;
        vout = vout == r->iv1 ? r->iv0 : r->iv1;
    }
    return hipGetLastError() == hipSuccess ? RL_OK : RL_EDEVICE;
}

extern "C" int rl_route_unpack(rl_router* r, size_t m, const uint32_t* slot, const rl_route_res* back,
                               uint8_t* decision, int64_t* remaining, int64_t* retry_after_ns, int64_t* reset_at_ns,
                               void* stream) {
    if (!r || m > r->max_batch ||
        (m && (!slot || !back || !decision || !remaining || !retry_after_ns || !reset_at_ns)))
        return RL_EINVAL;
    if (!m) return RL_OK;
    (void)hipSetDevice(r->device);
    // one request per thread: a wave reads 64 consecutive result records
    // when the slots increase (each owner's results come back in its
    // requests' order) -- 10 us per 1M requests in isolation, faster than
    // four per thread (14.5 us; profiles/r5m_route_unpack.txt)
    k_route_unpack<<<grid_for(m), RT_BLOCK, 0, (hipStream_t)stream>>>((uint32_t)m, slot, back, decision, remaining,
                                                                     retry_after_ns, reset_at_ns);
    return hipGetLastError() == hipSuccess ? RL_OK : RL_EDEVICE;
}
