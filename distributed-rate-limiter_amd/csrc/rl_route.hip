// rl_route.hip -- the routing kernels of include/rl_route.h: hash-sharded
// request batches across the GPUs of a node.
//
// All byte/integer work, HBM-bound, no MFMA:
//   pack     owner hash, per-tile owner counts, a one-block scan, a stable
//            scatter into per-owner groups of 32-byte records (ranks from wave
//            ballots, as rl_sort.h), so each group is one contiguous all-to-all
//            chunk
//   merge    the received records in arrival order at one shared store: by
//            arrival time (ties: source rank, source position), a record's
//            arrival time being the running max of ts over its source's
//            records so far (a server sends its requests in its own order, so
//            a source's order is always kept); a stable LSD radix sort of
//            (arrival - earliest) with as many 8-bit passes as the span needs
//            (rl_sort.h's one-sweep k_sort_pass, up to 48-bit keys; digit
//            histograms fused into the key kernels), then one gather into the
//            engine's input arrays
//   results  / unpack: 32-byte result records gathered by position, written
//            coalesced
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
constexpr int MERGE_PASSES = 6;                // arrival keys of up to 48 bits (spans < 78 h), 8-bit digits
constexpr int MERGE_KEY_BITS = 8 * MERGE_PASSES;

// router status bits (sticky, cleared by rl_router_sync)
constexpr uint32_t RS_SPAN = 1u;               // received ts span >= 2^48 ns

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

// summary of a batch (pack): earliest / latest ts (biased), whether ts ever decreases
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
    __shared__ uint32_t s_uns;
    __shared__ unsigned long long s_lo[RT_BLOCK / 64], s_hi[RT_BLOCK / 64];
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
        // a wave's 64 requests are consecutive: the predecessor's ts is the
        // lane below (lane 0 loads it)
        const uint32_t i = base + j * RT_BLOCK + threadIdx.x;
        const bool ok = i < m;
        const uint32_t own = ok ? owner_of(key[i], world) : 0u;
        const int64_t t = ok ? ts[i] : 0;
        int64_t tp = __shfl_up(t, 1);
        if (lane == 0) tp = (ok && i > 0) ? ts[i - 1] : t;
        // one LDS add per owner per wave (not per request: at small world
        // every request of a tile would hit one counter)
        const uint64_t peers = owner_peers(own, world, ok);
        if (ok && (peers & lt) == 0) atomicAdd(&s_cnt[own], (uint32_t)__popcll(peers));
        if (ok) {
            const unsigned long long b = bias(t);
            lo = b < lo ? b : lo;
            hi = b > hi ? b : hi;
            if (i > 0 && tp > t) uns = 1;
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
    if (uns) s_uns = 1;
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

// block o: owner o's output offset per tile (the requests of owners before o
// + an exclusive prefix over tiles) into tile_off, and owner o's info row
__global__ __launch_bounds__(RT_BLOCK) void k_route_scan(uint32_t tiles, uint32_t world,
                                                         const uint32_t* __restrict__ tile_cnt,
                                                         uint32_t* __restrict__ tile_off,
                                                         const PackSum* __restrict__ tile_sum,
                                                         int64_t* __restrict__ info) {
    __shared__ uint32_t s_tmp[RT_BLOCK / 64];
    __shared__ uint32_t s_run;
    __shared__ unsigned long long s_lo[RT_BLOCK / 64], s_hi[RT_BLOCK / 64];
    __shared__ uint32_t s_uns;
    const uint32_t o = blockIdx.x, tid = threadIdx.x;
    // the batch summary from the tiles' summaries
    unsigned long long lo = ~0ull, hi = 0;
    uint32_t uns = 0;
    for (uint32_t t = tid; t < tiles; t += RT_BLOCK) {
        const PackSum ps = tile_sum[t];
        lo = ps.lo < lo ? ps.lo : lo;
        hi = ps.hi > hi ? ps.hi : hi;
        uns |= ps.unsorted;
    }
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long l2 = __shfl_xor(lo, off), h2 = __shfl_xor(hi, off);
        lo = l2 < lo ? l2 : lo;
        hi = h2 > hi ? h2 : hi;
    }
    if (tid == 0) s_uns = 0;
    __syncthreads();
    if ((tid & 63) == 0) {
        s_lo[tid >> 6] = lo;
        s_hi[tid >> 6] = hi;
    }
    if (uns) s_uns = 1;   // benign race: every writer stores 1
    __syncthreads();
    uint32_t part = 0;
    for (uint32_t k = tid; k < tiles * o; k += RT_BLOCK) part += tile_cnt[(size_t)(k / o) * world + (k % o)];
    for (int off = 32; off > 0; off >>= 1) part += __shfl_xor(part, off);
    if ((tid & 63) == 0) s_tmp[tid >> 6] = part;
    __syncthreads();
    if (tid == 0) {
        uint32_t b = 0;
        for (int w = 0; w < RT_BLOCK / 64; w++) b += s_tmp[w];
        s_run = b;
    }
    __syncthreads();
    const uint32_t base = s_run;
    uint32_t run = base;
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
        row[0] = run - base;
        row[1] = tiles ? unbias(lo) : INT64_MAX;
        row[2] = tiles ? unbias(hi) : INT64_MIN;
        row[3] = s_uns ? 0 : 1;
    }
}

// stable scatter of the requests into per-owner groups
__global__ __launch_bounds__(RT_BLOCK) void k_route_scatter(uint32_t m, const uint64_t* __restrict__ key,
                                                            const int64_t* __restrict__ ts,
                                                            const int64_t* __restrict__ n,
                                                            const uint32_t* __restrict__ cfg, uint32_t world,
                                                            const uint32_t* __restrict__ tile_off,
                                                            rl_route_rec* __restrict__ send,
                                                            uint32_t* __restrict__ slot) {
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
#pragma unroll
    for (int j = 0; j < RT_ITEMS; j++) {
        const uint32_t i = base + j * 64 + lane;
        if (i >= m) continue;
        const uint32_t p = s_wcnt[wave][own[j]] + rank[j];
        rl_route_rec r;
        r.key = key[i];
        r.ts = ts[i];
        r.n = n[i];
        r.cfg = cfg[i];
        r.pos = i;
        send[p] = r;
        slot[i] = p;
    }
}

// The merge's plan, made on the host from the received info rows (the caller
// read them to size the record exchange): which kernels run at all
struct MergePlan {
    int64_t lo;         // time-key origin: earliest ts of any source that sent records
    int64_t clock;      // the store clock of the earlier steps (ms)
    uint32_t ident;     // at most one source sent records: received order is the decision order
    uint32_t scan;      // a source's batch is out of time order: arrival = running max of its ts
    uint32_t npass;     // 8-bit sort passes the arrival-key span needs (0 when ident)
};

// ctrl layout: digit histograms of the passes, one tile counter per pass, the
// sort's look-back flags; the passes' look-back status follows, npass x tiles
constexpr uint32_t MC_HIST = 0;
constexpr uint32_t MC_TILE = MC_HIST + MERGE_PASSES * RADIX;
constexpr uint32_t MC_SFLAGS = MC_TILE + MERGE_PASSES;
constexpr uint32_t MC_WORDS = (MC_SFLAGS + 1 + 63) & ~63u;
constexpr int MT_ITEMS = 4;                       // consecutive records per thread (merge scans)
constexpr uint32_t MT_TILE = RT_BLOCK * MT_ITEMS;
constexpr int SRC_BITS = 58;                      // composite key: source << 58 | (ts - lo)
constexpr uint64_t OFF_MASK = (1ull << SRC_BITS) - 1;

// source rank of received record i (sources are contiguous, in rank order)
__device__ inline uint64_t src_of(uint32_t i, const uint32_t* s_end, uint32_t world) {
    uint32_t s = 0;
    while (s + 1 < world && i >= s_end[s]) s++;
    return s;
}
__device__ inline void load_src_ends(const int64_t* __restrict__ info, uint32_t world, uint32_t* s_end) {
    if (threadIdx.x == 0) {
        uint64_t e = 0;
        for (uint32_t r = 0; r < world; r++) {
            e += (uint64_t)info[(size_t)RL_ROUTE_INFO * r];
            s_end[r] = (uint32_t)e;
        }
    }
    __syncthreads();
}
// a record's composite arrival key: (source << 58) | (ts - lo).  The running
// max of the composite along the received buffer restarts at every source
// (a later source's keys are larger), so it is each source's running max of
// ts -- the record's arrival time at the store
__device__ inline uint64_t composite(const rl_route_rec& r, uint64_t src, int64_t lo) {
    const uint64_t off = (uint64_t)(r.ts - lo);
    return (src << SRC_BITS) | (off & OFF_MASK);
}

// per tile of MT_TILE records: the max composite (scan inputs; plan.scan only)
__global__ __launch_bounds__(RT_BLOCK) void k_merge_tmax(uint32_t m, const rl_route_rec* __restrict__ rec,
                                                         const int64_t* __restrict__ info, uint32_t world,
                                                         MergePlan plan, unsigned long long* tmax) {
    __shared__ uint32_t s_end[MAX_WORLD];
    __shared__ unsigned long long s_w[RT_BLOCK / 64];
    load_src_ends(info, world, s_end);
    unsigned long long mx = 0;
#pragma unroll
    for (int q = 0; q < MT_ITEMS; q++) {
        const uint32_t i = blockIdx.x * MT_TILE + threadIdx.x * MT_ITEMS + q;
        if (i < m) {
            const unsigned long long c = composite(rec[i], src_of(i, s_end, world), plan.lo);
            mx = c > mx ? c : mx;
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

// exclusive running max over the tiles (one block; plan.scan only)
__global__ __launch_bounds__(1024) void k_merge_tscan(uint32_t tiles, unsigned long long* tmax) {
    __shared__ unsigned long long s_w[16];
    __shared__ unsigned long long s_carry;
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) s_carry = 0;
    __syncthreads();
    for (uint32_t t0 = 0; t0 < tiles; t0 += 1024) {
        const uint32_t t = t0 + tid;
        const unsigned long long v = t < tiles ? tmax[t] : 0ull;
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
        if (t < tiles) tmax[t] = ex;   // exclusive: the max of every earlier record
        if (tid == 1023) s_carry = inc > pre ? inc : pre;
        __syncthreads();
    }
}

// arrival key of every received record: kk[i] = (arrival time - lo), the
// running max of ts over its source's records so far (or ts itself when every
// source is in time order); with a sort (not ident), the sort's low 32-bit
// keys and the digit histograms of passes 0-3
__global__ __launch_bounds__(RT_BLOCK) void k_merge_keys(uint32_t m, const rl_route_rec* __restrict__ rec,
                                                         const int64_t* __restrict__ info, uint32_t world,
                                                         MergePlan plan, uint32_t* ctrl,
                                                         const unsigned long long* __restrict__ tpre,
                                                         unsigned long long* __restrict__ kk,
                                                         uint32_t* __restrict__ kout) {
    const bool ident = plan.ident != 0, scan = plan.scan != 0;
    __shared__ uint32_t s_end[MAX_WORLD];
    __shared__ uint32_t lh[4][RADIX];
    __shared__ unsigned long long s_w[RT_BLOCK / 64];
    for (int p = 0; p < 4; p++) lh[p][threadIdx.x] = 0;
    load_src_ends(info, world, s_end);
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t i0 = blockIdx.x * MT_TILE + threadIdx.x * MT_ITEMS;
    unsigned long long c[MT_ITEMS];
    unsigned long long run = 0;
#pragma unroll
    for (int q = 0; q < MT_ITEMS; q++) {
        const uint32_t i = i0 + q;
        c[q] = i < m ? composite(rec[i], src_of(i, s_end, world), plan.lo) : 0ull;
        if (scan) {
            run = c[q] > run ? c[q] : run;
            c[q] = run;                                  // inclusive within the thread
        }
    }
    if (scan) {
        // exclusive max over the earlier threads of the tile and the earlier tiles
        unsigned long long inc = run;
        for (int o = 1; o < 64; o <<= 1) {
            const unsigned long long u = __shfl_up(inc, o, 64);
            if (lane >= (uint32_t)o) inc = u > inc ? u : inc;
        }
        if (lane == 63) s_w[w] = inc;
        __syncthreads();
        unsigned long long pre = tpre[blockIdx.x];
        for (uint32_t k = 0; k < w; k++) pre = s_w[k] > pre ? s_w[k] : pre;
        unsigned long long ex = __shfl_up(inc, 1, 64);
        ex = lane ? (ex > pre ? ex : pre) : pre;
#pragma unroll
        for (int q = 0; q < MT_ITEMS; q++) c[q] = c[q] > ex ? c[q] : ex;
    }
    __syncthreads();   // lh zeroed
#pragma unroll
    for (int q = 0; q < MT_ITEMS; q++) {
        const uint32_t i = i0 + q;
        if (i >= m) continue;
        const unsigned long long off = c[q] & OFF_MASK;
        kk[i] = off;
        if (!ident) {
            const uint32_t k = (uint32_t)off;
            kout[i] = k;
#pragma unroll
            for (int p = 0; p < 4; p++) atomicAdd(&lh[p][(k >> (8 * p)) & (RADIX - 1)], 1u);
        }
    }
    __syncthreads();
    if (!ident)
        for (int p = 0; p < 4; p++) {
            const uint32_t v = lh[p][threadIdx.x];
            if (v) atomicAdd(&ctrl[MC_HIST + p * RADIX + threadIdx.x], v);
        }
}

// after four passes (data in kin/vin): the high 32 bits of the arrival keys
// as the next passes' keys, and their digit histograms (spans of 2^32 ns or more)
__global__ __launch_bounds__(RT_BLOCK) void k_merge_rekey(uint32_t m, uint32_t* ctrl,
                                                          const unsigned long long* __restrict__ kk,
                                                          uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin) {
    __shared__ uint32_t lh[MERGE_PASSES - 4][RADIX];
    for (int p = 0; p < MERGE_PASSES - 4; p++) lh[p][threadIdx.x] = 0;
    __syncthreads();
    for (uint32_t i = blockIdx.x * RT_BLOCK + threadIdx.x; i < m; i += gridDim.x * RT_BLOCK) {
        const uint32_t k = (uint32_t)(kk[vin[i]] >> 32);
        kin[i] = k;
#pragma unroll
        for (int p = 0; p < MERGE_PASSES - 4; p++) atomicAdd(&lh[p][(k >> (8 * p)) & (RADIX - 1)], 1u);
    }
    __syncthreads();
    for (int p = 0; p < MERGE_PASSES - 4; p++) {
        const uint32_t v = lh[p][threadIdx.x];
        if (v) atomicAdd(&ctrl[MC_HIST + (4 + p) * RADIX + threadIdx.x], v);
    }
}

// sorted position p holds received record v[p] (identity when ident): the
// engine's inputs in order, with the store clock max(floor(arrival / 1e6),
// clock of earlier steps)
__global__ __launch_bounds__(RT_BLOCK) void k_merge_gather(uint32_t m, MergePlan plan, const uint32_t* __restrict__ v,
                                                           const rl_route_rec* __restrict__ rec,
                                                           const unsigned long long* __restrict__ kk,
                                                           uint64_t* __restrict__ key, int64_t* __restrict__ ts,
                                                           int64_t* __restrict__ n, uint32_t* __restrict__ cfg,
                                                           int64_t* __restrict__ sms, uint32_t* __restrict__ at) {
    const bool ident = plan.ident != 0, keyed = !ident || plan.scan != 0;
    const int64_t c0 = plan.clock;
    for (uint32_t p = blockIdx.x * RT_BLOCK + threadIdx.x; p < m; p += gridDim.x * RT_BLOCK) {
        const uint32_t i = ident ? p : v[p];
        const rl_route_rec r = rec[i];
        key[p] = r.key;
        ts[p] = r.ts;
        n[p] = r.n;
        cfg[p] = r.cfg;
        const int64_t arrive = keyed ? (int64_t)((uint64_t)plan.lo + kk[i]) : r.ts;
        const int64_t ms = floor_div(arrive, 1000000LL);
        sms[p] = ms > c0 ? ms : c0;
        at[i] = p;
    }
}

// ---- the single-source merge planned on the device (world 1) ----------------
// One source: the received order is the decision order, and a request arrives
// at the running max of ts so far (= ts when the batch is in time order).  No
// host reads anything: a per-tile max, one scan block that also advances the
// store clock (a device word: the merges run in step order), one gather.
constexpr unsigned long long TS_BIAS = 1ull << 63;   // int64 order as uint64 order

__global__ __launch_bounds__(RT_BLOCK) void k_m1_tmax(uint32_t m, const rl_route_rec* __restrict__ rec,
                                                      unsigned long long* tmax) {
    __shared__ unsigned long long s_w[RT_BLOCK / 64];
    unsigned long long mx = 0;
#pragma unroll
    for (int q = 0; q < MT_ITEMS; q++) {
        const uint32_t i = blockIdx.x * MT_TILE + threadIdx.x * MT_ITEMS + q;
        if (i < m) {
            const unsigned long long c = (unsigned long long)rec[i].ts ^ TS_BIAS;
            mx = c > mx ? c : mx;
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

// exclusive running max over the tiles (in place); then tmax[tiles] = the
// clock of the earlier steps (for the gather) and the clock advances to
// max(clock, floor(latest ts / 1e6)) -- what the host plan does with the info rows
__global__ __launch_bounds__(1024) void k_m1_tscan(uint32_t tiles, unsigned long long* tmax, int64_t* clock) {
    __shared__ unsigned long long s_w[16];
    __shared__ unsigned long long s_carry;
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) s_carry = 0;
    __syncthreads();
    for (uint32_t t0 = 0; t0 < tiles; t0 += 1024) {
        const uint32_t t = t0 + tid;
        const unsigned long long v = t < tiles ? tmax[t] : 0ull;
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
        if (t < tiles) tmax[t] = ex;
        if (tid == 1023) s_carry = inc > pre ? inc : pre;
        __syncthreads();
    }
    if (tid == 0) {
        const int64_t c0 = *clock;
        tmax[tiles] = (unsigned long long)c0;
        const int64_t ms = floor_div((int64_t)(s_carry ^ TS_BIAS), 1000000LL);
        *clock = ms > c0 ? ms : c0;
    }
}

// the engine's inputs in received order, server clock from the running max
__global__ __launch_bounds__(RT_BLOCK) void k_m1_gather(uint32_t m, uint32_t tiles, const rl_route_rec* __restrict__ rec,
                                                        const unsigned long long* __restrict__ tpre,
                                                        uint64_t* __restrict__ key, int64_t* __restrict__ ts,
                                                        int64_t* __restrict__ n, uint32_t* __restrict__ cfg,
                                                        int64_t* __restrict__ sms, uint32_t* __restrict__ at) {
    __shared__ unsigned long long s_w[RT_BLOCK / 64];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t i0 = blockIdx.x * MT_TILE + threadIdx.x * MT_ITEMS;
    const int64_t c0 = (int64_t)tpre[tiles];
    rl_route_rec r[MT_ITEMS];
    unsigned long long c[MT_ITEMS];
    unsigned long long run = 0;
#pragma unroll
    for (int q = 0; q < MT_ITEMS; q++) {
        const uint32_t i = i0 + q;
        if (i < m) r[q] = rec[i];
        c[q] = i < m ? (unsigned long long)r[q].ts ^ TS_BIAS : 0ull;
        run = c[q] > run ? c[q] : run;
        c[q] = run;                                  // inclusive within the thread
    }
    unsigned long long inc = run;
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long u = __shfl_up(inc, o, 64);
        if (lane >= (uint32_t)o) inc = u > inc ? u : inc;
    }
    if (lane == 63) s_w[w] = inc;
    __syncthreads();
    unsigned long long pre = tpre[blockIdx.x];
    for (uint32_t k = 0; k < w; k++) pre = s_w[k] > pre ? s_w[k] : pre;
    unsigned long long ex = __shfl_up(inc, 1, 64);
    ex = lane ? (ex > pre ? ex : pre) : pre;
#pragma unroll
    for (int q = 0; q < MT_ITEMS; q++) {
        const uint32_t i = i0 + q;
        if (i >= m) continue;
        const unsigned long long a = c[q] > ex ? c[q] : ex;
        const int64_t ms = floor_div((int64_t)(a ^ TS_BIAS), 1000000LL);
        key[i] = r[q].key;
        ts[i] = r[q].ts;
        n[i] = r[q].n;
        cfg[i] = r[q].cfg;
        sms[i] = ms > c0 ? ms : c0;
        at[i] = i;
    }
}

__global__ __launch_bounds__(RT_BLOCK) void k_route_results(uint32_t m, const uint32_t* __restrict__ at,
                                                            const uint8_t* __restrict__ dec,
                                                            const int64_t* __restrict__ rem,
                                                            const int64_t* __restrict__ retry,
                                                            const int64_t* __restrict__ reset,
                                                            rl_route_res* __restrict__ res) {
    for (uint32_t i = blockIdx.x * RT_BLOCK + threadIdx.x; i < m; i += gridDim.x * RT_BLOCK) {
        const uint32_t p = at[i];
        res[i] = rl_route_res{(int64_t)dec[p], rem[p], retry[p], reset[p]};
    }
}

__global__ __launch_bounds__(RT_BLOCK) void k_route_unpack(uint32_t m, const uint32_t* __restrict__ slot,
                                                           const rl_route_res* __restrict__ back,
                                                           uint8_t* __restrict__ dec, int64_t* __restrict__ rem,
                                                           int64_t* __restrict__ retry,
                                                           int64_t* __restrict__ reset) {
    for (uint32_t i = blockIdx.x * RT_BLOCK + threadIdx.x; i < m; i += gridDim.x * RT_BLOCK) {
        const rl_route_res r = back[slot[i]];
        dec[i] = (uint8_t)r.decision;
        rem[i] = r.remaining;
        retry[i] = r.retry_after_ns;
        reset[i] = r.reset_at_ns;
    }
}

// one GPU: nothing travels between the owner's results and the sender's
// unpack, so the caller's outputs come straight from the engine's: request i
// was received as send slot[i] and decided at position at[slot[i]]
__global__ __launch_bounds__(RT_BLOCK) void k_route_results_local(uint32_t m, const uint32_t* __restrict__ slot,
                                                                  const uint32_t* __restrict__ at,
                                                                  const uint8_t* __restrict__ dec_in,
                                                                  const int64_t* __restrict__ rem_in,
                                                                  const int64_t* __restrict__ retry_in,
                                                                  const int64_t* __restrict__ reset_in,
                                                                  uint8_t* __restrict__ dec, int64_t* __restrict__ rem,
                                                                  int64_t* __restrict__ retry,
                                                                  int64_t* __restrict__ reset) {
    for (uint32_t i = blockIdx.x * RT_BLOCK + threadIdx.x; i < m; i += gridDim.x * RT_BLOCK) {
        const uint32_t p = at[slot[i]];
        dec[i] = dec_in[p];
        rem[i] = rem_in[p];
        retry[i] = retry_in[p];
        reset[i] = reset_in[p];
    }
}

int grid_for(size_t m) { return (int)std::min<size_t>((m + RT_BLOCK - 1) / RT_BLOCK, 2048); }

}  // namespace

struct rl_router {
    int device = 0;
    uint32_t world = 1, max_batch = 0, max_recv = 0;
    uint32_t* tile_cnt = nullptr;    // pack: [tiles][world]
    uint32_t* tile_off = nullptr;    // pack: [tiles][world] output offsets
    PackSum* psum = nullptr;         // pack: per-tile summaries [tiles]
    uint32_t* ctrl = nullptr;        // merge: MC_* words + look-back status
    uint32_t* status = nullptr;      // merge: [npass][tiles][RADIX] of the current step
    uint32_t *k0 = nullptr, *k1 = nullptr, *v0 = nullptr, *v1 = nullptr;
    unsigned long long* kk = nullptr;     // merge: arrival key (arrival - lo) per received record
    unsigned long long* tmax = nullptr;   // merge: per-tile running-max scan
    uint32_t* d_status = nullptr;    // sticky router status: the sort's look-back flags
    uint32_t host_status = 0;        // sticky router status found by the host plan (RS_*)
    int64_t clock = INT64_MIN;        // the store clock of the next step (ms), kept in enqueue order
    int64_t* d_clock = nullptr;       // the same, on the device, for merges planned there (world 1)
    bool clock_on_device = false;     // a device-planned merge has run: the clock lives in d_clock
};

extern "C" int rl_router_create(int32_t device, int32_t world, uint32_t max_batch, uint32_t max_recv,
                                rl_router** out) {
    if (!out || world < 1 || world > MAX_WORLD || max_batch == 0 || max_recv == 0 || max_batch > (1u << 30) ||
        max_recv > (1u << 30))
        return RL_EINVAL;
    *out = nullptr;
    if (hipSetDevice(device) != hipSuccess) return RL_EDEVICE;
    rl_router* r = new rl_router();
    r->device = device;
    r->world = (uint32_t)world;
    r->max_batch = max_batch;
    r->max_recv = max_recv;
    const size_t ptiles = (max_batch + RT_TILE - 1) / RT_TILE;
    const size_t stiles = (max_recv + SORT_TILE - 1) / SORT_TILE;
    bool ok = hipMalloc(&r->tile_cnt, 4 * ptiles * world) == hipSuccess;
    ok = ok && hipMalloc(&r->tile_off, 4 * ptiles * world) == hipSuccess;
    ok = ok && hipMalloc(&r->psum, sizeof(PackSum) * (ptiles ? ptiles : 1)) == hipSuccess;
    ok = ok && hipMalloc(&r->ctrl, 4 * (MC_WORDS + (size_t)MERGE_PASSES * stiles * RADIX)) == hipSuccess;
    for (uint32_t** p : {&r->k0, &r->k1, &r->v0, &r->v1}) ok = ok && hipMalloc(p, 4 * (size_t)max_recv) == hipSuccess;
    ok = ok && hipMalloc(&r->kk, 8 * (size_t)max_recv) == hipSuccess;
    ok = ok && hipMalloc(&r->tmax, 8 * ((size_t)max_recv / MT_TILE + 2)) == hipSuccess;
    ok = ok && hipMalloc(&r->d_clock, 8) == hipSuccess;
    ok = ok && hipMalloc(&r->d_status, 4) == hipSuccess && hipMemset(r->d_status, 0, 4) == hipSuccess;
    if (!ok) {
        rl_router_destroy(r);
        return RL_ENOMEM;
    }
    r->status = r->ctrl + MC_WORDS;
    *out = r;
    return RL_OK;
}

extern "C" int rl_router_destroy(rl_router* r) {
    if (!r) return RL_EINVAL;
    (void)hipSetDevice(r->device);
    for (void* p : {(void*)r->tile_cnt, (void*)r->ctrl, (void*)r->k0, (void*)r->k1, (void*)r->v0, (void*)r->v1,
                    (void*)r->kk, (void*)r->tmax, (void*)r->d_clock,
                    (void*)r->d_status, (void*)r->tile_off, (void*)r->psum})
        (void)hipFree(p);
    delete r;
    return RL_OK;
}

extern "C" int rl_router_sync(rl_router* r, void* stream) {
    if (!r) return RL_EINVAL;
    (void)hipSetDevice(r->device);
    if (hipStreamSynchronize((hipStream_t)stream) != hipSuccess) return RL_EDEVICE;
    uint32_t s = 0;
    if (hipMemcpy(&s, r->d_status, 4, hipMemcpyDeviceToHost) != hipSuccess) return RL_EDEVICE;
    if (hipMemset(r->d_status, 0, 4) != hipSuccess) return RL_EDEVICE;
    const uint32_t h = r->host_status;
    r->host_status = 0;
    if (s & EF_LOOKBACK) return RL_ETIMEOUT;
    if (h & RS_SPAN) return RL_EINVAL;
    return RL_OK;
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
    k_route_scan<<<r->world, RT_BLOCK, 0, s>>>(tiles, r->world, r->tile_cnt, r->tile_off, r->psum, send_info);
    if (!m) return hipGetLastError() == hipSuccess ? RL_OK : RL_EDEVICE;
    k_route_scatter<<<tiles, RT_BLOCK, 0, s>>>((uint32_t)m, key, ts, n, cfg, r->world, r->tile_off, send, slot);
    return hipGetLastError() == hipSuccess ? RL_OK : RL_EDEVICE;
}

__global__ void k_merge_status(const uint32_t* sort_flags, uint32_t* status) {
    const uint32_t f = *sort_flags & EF_LOOKBACK;
    if (f) atomicOr(status, f);
}

extern "C" int rl_route_merge(rl_router* r, size_t m_recv, const rl_route_rec* recv, const int64_t* recv_info,
                              const int64_t* recv_info_host, uint64_t* key, int64_t* ts, int64_t* n, uint32_t* cfg,
                              int64_t* server_ms, uint32_t* at, void* stream) {
    if (!r || !recv_info || m_recv > r->max_recv || (m_recv && (!recv || !key || !ts || !n || !cfg || !server_ms || !at)))
        return RL_EINVAL;
    (void)hipSetDevice(r->device);
    hipStream_t s = (hipStream_t)stream;
    if (!recv_info_host) {
        // planned on the device: one source only (world 1), nothing read by the host
        if (r->world != 1) return RL_EINVAL;
        if (!r->clock_on_device) {
            if (hipMemcpyAsync(r->d_clock, &r->clock, 8, hipMemcpyHostToDevice, s) != hipSuccess) return RL_EDEVICE;
            if (hipStreamSynchronize(s) != hipSuccess) return RL_EDEVICE;
            r->clock_on_device = true;
        }
        const uint32_t m = (uint32_t)m_recv;
        if (!m) return RL_OK;
        const uint32_t mtiles = (m + MT_TILE - 1) / MT_TILE;
        k_m1_tmax<<<mtiles, RT_BLOCK, 0, s>>>(m, recv, r->tmax);
        k_m1_tscan<<<1, 1024, 0, s>>>(mtiles, r->tmax, r->d_clock);
        k_m1_gather<<<mtiles, RT_BLOCK, 0, s>>>(m, mtiles, recv, r->tmax, key, ts, n, cfg, server_ms, at);
        return hipGetLastError() == hipSuccess ? RL_OK : RL_EDEVICE;
    }
    if (r->clock_on_device) return RL_EINVAL;   // the clock is the device's now: keep planning there
    // the plan, on the host: the time-key origin and span of the sources that
    // sent records, whether a source is out of time order, the passes
    int64_t lo = INT64_MAX, hi = INT64_MIN, clock_next = r->clock;
    uint32_t sources = 0, sorted = 1;
    for (uint32_t q = 0; q < r->world; q++) {
        const int64_t* row = recv_info_host + (size_t)RL_ROUTE_INFO * q;
        if (row[2] != INT64_MIN) {   // after this step: clock = max(clock, floor(latest ts / 1e6))
            const int64_t ms = floor_div(row[2], 1000000LL);
            clock_next = ms > clock_next ? ms : clock_next;
        }
        if (row[0] == 0) continue;
        sources++;
        sorted &= row[3] != 0;
        lo = row[1] < lo ? row[1] : lo;
        hi = row[2] > hi ? row[2] : hi;
    }
    MergePlan plan{lo, r->clock, sources <= 1 ? 1u : 0u, sorted ? 0u : 1u, 0u};
    r->clock = clock_next;
    const uint32_t m = (uint32_t)m_recv;
    if (!m) return RL_OK;
    const uint64_t span = (uint64_t)hi - (uint64_t)lo;
    if (span >> MERGE_KEY_BITS) r->host_status |= RS_SPAN;
    if (!plan.ident) {
        plan.npass = 1;
        while (plan.npass < (uint32_t)MERGE_PASSES && (span >> (8 * plan.npass))) plan.npass++;
    }
    const uint32_t mtiles = (m + MT_TILE - 1) / MT_TILE;
    const uint32_t stiles = (m + SORT_TILE - 1) / SORT_TILE;
    if (!plan.ident || plan.scan) {
        // the control words and the look-back status of the passes this step runs
        const size_t words = MC_WORDS + (size_t)plan.npass * stiles * RADIX;
        if (hipMemsetAsync(r->ctrl, 0, 4 * words, s) != hipSuccess) return RL_EDEVICE;
        if (plan.scan) {
            k_merge_tmax<<<mtiles, RT_BLOCK, 0, s>>>(m, recv, recv_info, r->world, plan, r->tmax);
            k_merge_tscan<<<1, 1024, 0, s>>>(mtiles, r->tmax);
        }
        k_merge_keys<<<mtiles, RT_BLOCK, 0, s>>>(m, recv, recv_info, r->world, plan, r->ctrl, r->tmax, r->kk, r->k0);
    }
    uint32_t* sflags = r->ctrl + MC_SFLAGS;
    uint32_t *kin = r->k0, *vin = r->v0, *kout = r->k1, *vout = r->v1;
    for (uint32_t p = 0; p < plan.npass; p++) {
        uint32_t* st = r->status + (size_t)p * stiles * RADIX;
        if (p == 4) k_merge_rekey<<<grid_for(m), RT_BLOCK, 0, s>>>(m, r->ctrl, r->kk, kin, vin);
        if (p == 0)
            k_sort_pass<true><<<stiles, SORT_BLOCK, 0, s>>>(kin, vin, kout, vout, m, 0, r->ctrl + MC_HIST, st,
                                                            r->ctrl + MC_TILE, sflags);
        else
            k_sort_pass<false><<<stiles, SORT_BLOCK, 0, s>>>(kin, vin, kout, vout, m, 8 * (p & 3),
                                                             r->ctrl + MC_HIST + p * RADIX, st, r->ctrl + MC_TILE + p,
                                                             sflags);
        std::swap(kin, kout);
        std::swap(vin, vout);
    }
    k_merge_gather<<<grid_for(m), RT_BLOCK, 0, s>>>(m, plan, vin, recv, r->kk, key, ts, n, cfg, server_ms, at);
    if (plan.npass) k_merge_status<<<1, 1, 0, s>>>(sflags, r->d_status);
    return hipGetLastError() == hipSuccess ? RL_OK : RL_EDEVICE;
}

extern "C" int rl_route_results(size_t m_recv, const uint32_t* at, const uint8_t* decision, const int64_t* remaining,
                                const int64_t* retry_after_ns, const int64_t* reset_at_ns, rl_route_res* res,
                                void* stream) {
    if (m_recv > (1u << 30) || (m_recv && (!at || !decision || !remaining || !retry_after_ns || !reset_at_ns || !res)))
        return RL_EINVAL;
    if (!m_recv) return RL_OK;
    k_route_results<<<grid_for(m_recv), RT_BLOCK, 0, (hipStream_t)stream>>>((uint32_t)m_recv, at, decision, remaining,
                                                                            retry_after_ns, reset_at_ns, res);
    return hipGetLastError() == hipSuccess ? RL_OK : RL_EDEVICE;
}

extern "C" int rl_route_unpack(size_t m, const uint32_t* slot, const rl_route_res* back, uint8_t* decision,
                               int64_t* remaining, int64_t* retry_after_ns, int64_t* reset_at_ns, void* stream) {
    if (m > (1u << 30) || (m && (!slot || !back || !decision || !remaining || !retry_after_ns || !reset_at_ns)))
        return RL_EINVAL;
    if (!m) return RL_OK;
    k_route_unpack<<<grid_for(m), RT_BLOCK, 0, (hipStream_t)stream>>>((uint32_t)m, slot, back, decision, remaining,
                                                                      retry_after_ns, reset_at_ns);
    return hipGetLastError() == hipSuccess ? RL_OK : RL_EDEVICE;
}

extern "C" int rl_route_results_local(size_t m, const uint32_t* slot, const uint32_t* at, const uint8_t* decision_in,
                                      const int64_t* remaining_in, const int64_t* retry_in, const int64_t* reset_in,
                                      uint8_t* decision, int64_t* remaining, int64_t* retry_after_ns,
                                      int64_t* reset_at_ns, void* stream) {
    if (m > (1u << 30) || (m && (!slot || !at || !decision_in || !remaining_in || !retry_in || !reset_in || !decision ||
                                 !remaining || !retry_after_ns || !reset_at_ns)))
        return RL_EINVAL;
    if (!m) return RL_OK;
    k_route_results_local<<<grid_for(m), RT_BLOCK, 0, (hipStream_t)stream>>>(
        (uint32_t)m, slot, at, decision_in, remaining_in, retry_in, reset_in, decision, remaining, retry_after_ns,
        reset_at_ns);
    return hipGetLastError() == hipSuccess ? RL_OK : RL_EDEVICE;
}
