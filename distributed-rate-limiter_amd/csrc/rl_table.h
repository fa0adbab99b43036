// rl_table.h -- HBM-resident open-addressing per-key state tables.
//
// Replaces the Redis keyspace the reference scripts touch:
//   token bucket : one hash per user key "P:k" {tokens, last_refill} + TTL
//                  (tokenbucket.go:31,48-49)
//   window counts: string keys "P:k:ws" + TTL (fixedwindow.go:22-24,
//                  slidingwindow.go:23-28); the two live windows of a user key
//                  share one 64-byte entry so SW's curr/prev pair is one line.
// Layout: array-of-structs, one entry per slot, entry size = a power of two
// that divides the 128-byte line, so a probe hit brings the state with it.
// Linear probing on a 64-bit mix of the key id; keys are only ever inserted
// (EMPTY -> id by CAS), never moved, so a stale EMPTY read is harmless: the CAS
// resolves it.
#pragma once

#include "rl_semantics.h"

namespace rl {

struct alignas(32) TbEntry {
    uint64_t key;
    double tok;      // stored `tokens`, already tostring/tonumber round-tripped
    double last;     // stored `last_refill`
    int64_t when;    // expiry (server ms), ABSENT if the key does not exist
};
static_assert(sizeof(TbEntry) == 32, "TbEntry must be 32 bytes");

struct alignas(64) WinEntry {
    uint64_t key;
    int64_t nspill;  // this user key's entries in the spill table (rl_window.h)
    WinSlot s[2];
};
static_assert(sizeof(WinEntry) == 64, "WinEntry must be 64 bytes");

// The rest of the window keyspace.  Redis keeps any number of live window
// keys "B:ws" per user key B (fixedwindow.go:72-75, slidingwindow.go:74-79);
// the 2-slot entry holds the two newest, and a live key that has to leave it
// (or an older window key created out of order) lives here.  Open addressing
// by the USER key with linear probing from spill_home(k): every spill entry
// of k sits before the first never-used slot of k's probe sequence (key ids
// are never removed), and only k's segment -- one thread or one wave of one
// replay -- touches them, so k reuses its own dead entries without races.
struct alignas(32) SpillEntry {
    uint64_t key;    // user key id (EMPTY_KEY: never used)
    int64_t ws;      // window start (Unix s)
    int64_t cnt;
    int64_t when;    // expiry (server ms); ABSENT: deleted (the slot stays k's)
};
static_assert(sizeof(SpillEntry) == 32, "SpillEntry must be 32 bytes");

struct Spill {
    SpillEntry* tab;
    uint64_t mask;
};

RL_HD inline uint64_t mix64(uint64_t x) {
    x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ULL;
    x ^= x >> 27; x *= 0x94d049bb133111ebULL;
    x ^= x >> 31; return x;
}

constexpr uint32_t NO_SLOT = 0xffffffffu;
// probe-length bound: a longer run means the table is (effectively) full
constexpr uint64_t MAX_PROBES = 1u << 13;

// find-or-insert `k` in a table whose entries are `stride` bytes with the key
// in the first 8 bytes; returns the slot or NO_SLOT when the table is full.
template <typename E>
__device__ inline uint32_t probe_insert(E* tab, uint64_t mask, uint64_t k) {
    uint64_t h = mix64(k) & mask;
    const uint64_t lim = mask < MAX_PROBES ? mask : MAX_PROBES;
    for (uint64_t p = 0; p <= lim; p++) {
        uint64_t* kp = &tab[h].key;
        uint64_t cur = *kp;
        if (cur == k) return (uint32_t)h;
        if (cur == EMPTY_KEY) {
            unsigned long long prev = atomicCAS((unsigned long long*)kp, (unsigned long long)EMPTY_KEY,
                                                (unsigned long long)k);
            if (prev == EMPTY_KEY || prev == k) return (uint32_t)h;
        }
        h = (h + 1) & mask;
    }
    return NO_SLOT;
}

// probe_insert with the first probe's key word already loaded (`cur`, the
// key at slot h = mix64(k) & mask): lets a thread issue the first loads of
// several requests before resolving any (memory-level parallelism)
// (*ins: this call's CAS inserted the key -- its entry holds the initial,
// absent state: keys are never removed from a table, only rehashed by GC)
template <typename E>
__device__ inline uint32_t probe_insert_at(E* tab, uint64_t mask, uint64_t k, uint64_t h, uint64_t cur,
                                          bool* ins = nullptr) {
    const uint64_t lim = mask < MAX_PROBES ? mask : MAX_PROBES;
    for (uint64_t p = 0; p <= lim; p++) {
        if (p) cur = tab[h].key;
        if (cur == k) return (uint32_t)h;
        if (cur == EMPTY_KEY) {
            unsigned long long prev = atomicCAS((unsigned long long*)&tab[h].key, (unsigned long long)EMPTY_KEY,
                                                (unsigned long long)k);
            if (prev == EMPTY_KEY || prev == k) {
                if (ins) *ins = prev == EMPTY_KEY;
                return (uint32_t)h;
            }
        }
        h = (h + 1) & mask;
    }
    return NO_SLOT;
}

// lookup only (Reset path)
template <typename E>
__device__ inline uint32_t probe_find(const E* tab, uint64_t mask, uint64_t k) {
    uint64_t h = mix64(k) & mask;
    const uint64_t lim = mask < MAX_PROBES ? mask : MAX_PROBES;
    for (uint64_t p = 0; p <= lim; p++) {
        uint64_t cur = tab[h].key;
        if (cur == k) return (uint32_t)h;
        if (cur == EMPTY_KEY) return NO_SLOT;
        h = (h + 1) & mask;
    }
    return NO_SLOT;
}

// Liveness at server clock now_ms, as Redis's expiry sees it: a token-bucket
// entry is its hash key; a window entry holds up to two counter keys and lives
// while either does (lazy expiry would treat the others as absent anyway).
__device__ inline bool entry_live(const TbEntry& x, int64_t now_ms, int32_t profile) {
    return x.key != EMPTY_KEY && x.when != ABSENT && key_alive(x.when, now_ms, profile);
}
__device__ inline bool entry_live(const WinEntry& x, int64_t now_ms, int32_t profile) {
    if (x.key == EMPTY_KEY) return false;
    for (int k = 0; k < 2; k++)
        if (x.s[k].when != ABSENT && key_alive(x.s[k].when, now_ms, profile)) return true;
    return false;
}
__device__ inline bool entry_live(const SpillEntry& x, int64_t now_ms, int32_t profile) {
    return x.key != EMPTY_KEY && x.when != ABSENT && key_alive(x.when, now_ms, profile);
}

// what table GC keeps: a window entry also stays while its user key has
// spill entries (their liveness is recounted by k_spill_rehash)
__device__ inline bool entry_kept(const TbEntry& x, int64_t now_ms, int32_t profile) {
    return entry_live(x, now_ms, profile);
}
__device__ inline bool entry_kept(const WinEntry& x, int64_t now_ms, int32_t profile) {
    return x.key != EMPTY_KEY && (x.nspill > 0 || entry_live(x, now_ms, profile));
}
__device__ inline void gc_copy(TbEntry& dst, const TbEntry& x) { dst = x; }
__device__ inline void gc_copy(WinEntry& dst, const WinEntry& x) {
    WinEntry y = x;
    y.nspill = 0;   // recounted from the live spill entries
    dst = y;
}

// Table GC / resize (rl_table_gc): re-insert every live entry of `old` into
// the empty table `nu`.  Keys are distinct, so concurrent inserts never race
// on one key.  counters[0] += live entries, counters[1] += entries that found
// no slot (the new table is too small: the caller keeps the old one).
template <typename E>
__global__ void k_rehash(const E* __restrict__ old, uint64_t n_old, E* nu, uint64_t mask_new, int64_t now_ms,
                         int32_t profile, unsigned long long* counters) {
    unsigned long long live = 0, lost = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n_old;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const E x = old[i];
        if (!entry_kept(x, now_ms, profile)) continue;
        live++;
        const uint32_t s = probe_insert(nu, mask_new, x.key);
        if (s == NO_SLOT) { lost++; continue; }
        gc_copy(nu[s], x);
    }
    if (live) atomicAdd(&counters[0], live);
    if (lost) atomicAdd(&counters[1], lost);
}

__device__ inline uint64_t spill_home(uint64_t k, uint64_t mask) { return mix64(k ^ 0x5bd1e9955bd1e995ULL) & mask; }

// occupied and live entries (rl_table_info_get)
template <typename E>
__global__ void k_table_count(const E* __restrict__ t, uint64_t n, int64_t now_ms, int32_t profile,
                              unsigned long long* counters) {
    unsigned long long used = 0, live = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const E x = t[i];
        used += x.key != EMPTY_KEY;
        live += entry_live(x, now_ms, profile);
    }
    if (used) atomicAdd(&counters[0], used);
    if (live) atomicAdd(&counters[1], live);
}

}  // namespace rl
