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
    int64_t pad;
    WinSlot s[2];
};
static_assert(sizeof(WinEntry) == 64, "WinEntry must be 64 bytes");

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

}  // namespace rl
