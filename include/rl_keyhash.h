/*
 * rl_keyhash.h -- on-GPU key formatting + hashing.
 *
 * The reference names every Redis key with string building on the host:
 *   Config.FormatKey            config.go:81-87     prefix + ":" + key ("" -> key)
 *   tokenBucketLimiter.AllowN   tokenbucket.go:95   redisKey := t.config.FormatKey(key)
 *   fixedWindowLimiter.formatKey fixedwindow.go:139-141  Sprintf("%s:%d", FormatKey(key), ws)
 *   slidingWindowLimiter.formatKey slidingwindow.go:150-152
 * Redis then looks the string up in its keyspace.  Here the window suffix is
 * already handled by the engine (state entries keyed by the base key carry
 * their window ids), so the only string work left is FormatKey plus the
 * keyspace lookup.  These entry points take a batch of raw user keys (one
 * concatenated byte buffer + offsets), form `prefix ":" key` on the device and
 * hash it with XXH64 (seed = the limiter's namespace), producing the key_id
 * array rl_decide_batch[_device] consumes (include/rl_engine.h).
 *
 *   key_id[i] = XXH64(FormatKey(prefix, bytes[offsets[i] .. offsets[i+1])), seed)
 *               (RL_KEY_RESERVED is mapped to RL_KEY_RESERVED - 1)
 *
 * Identity: distinct formatted keys share state only on a 64-bit hash
 * collision (probability ~ k^2 / 2^65 over k live keys: 3e-8 at 1M keys,
 * 2.7e-2 at 1e9).  Callers that need exact identity at 1e9 keys keep the
 * host interner of include/rl_limiter.h.
 *
 * Errors: RL_EINVAL for a prefix longer than RL_KEYHASH_MAX_PREFIX bytes, a
 * NULL array with m > 0, or (host entry point) offsets that decrease or run
 * past nbytes.  The device entry point cannot check offsets without a sync:
 * a request whose offsets are out of order or past nbytes gets
 * RL_KEY_RESERVED, which rl_decide_batch reports as RL_INVALID.
 */
#ifndef RL_KEYHASH_H
#define RL_KEYHASH_H

#include <stddef.h>
#include <stdint.h>

#include "rl_engine.h"

#ifdef __cplusplus
extern "C" {
#endif

#define RL_KEYHASH_MAX_PREFIX 240
/* largest m per call: the launch grid is a 32-bit work-item count */
#define RL_KEYHASH_MAX_KEYS ((uint64_t)0xFFFFFF00u)

/* The seed the engine's raw-key entry point hashes request i with: the
 * caller's seed with the request's config id mixed in, so each registered
 * config is its own key namespace (config 0 keeps the seed).  Two configs
 * never share state for one raw key -- a limiter instance owns its keys
 * (DESIGN.md §1). */
#define RL_CFG_SEED(seed, cfg_id) ((uint64_t)(seed) ^ ((uint64_t)(uint32_t)(cfg_id) * 0x9E3779B97F4A7C15ull))
static inline uint64_t rl_cfg_seed(uint64_t seed, uint32_t cfg_id) { return RL_CFG_SEED(seed, cfg_id); }

/* Device arrays, enqueued on `stream` (a hipStream_t; NULL = the null stream).
 * bytes: nbytes readable bytes; offsets: m + 1 entries. */
int rl_hash_keys_device(size_t m, const uint8_t* bytes, uint64_t nbytes, const uint64_t* offsets,
                        uint64_t seed, const char* prefix, size_t prefix_len, uint64_t* key_id,
                        void* stream);

/* The same ids computed on the host CPU (a server's per-request path, where a
 * GPU launch per key would cost more than the hash): cfg_id nullable -- when
 * given, request i is hashed with rl_cfg_seed(seed, cfg_id[i]) as
 * rl_decide_batch_keys_device does.  Offsets as rl_hash_keys. */
int rl_hash_keys_host(size_t m, const uint8_t* bytes, uint64_t nbytes, const uint64_t* offsets, uint64_t seed,
                      const uint32_t* cfg_id, const char* prefix, size_t prefix_len, uint64_t* key_id);

/* Host arrays on device `device`: copies in, hashes, copies out.  Synchronous. */
int rl_hash_keys(int32_t device, size_t m, const uint8_t* bytes, uint64_t nbytes, const uint64_t* offsets,
                 uint64_t seed, const char* prefix, size_t prefix_len, uint64_t* key_id);

/* rl_decide_batch_device (include/rl_engine.h) with raw keys instead of key
 * ids: the hashing above runs on the engine's grouping stream ahead of the
 * table probe, so batches stay pipelined (RL_OPT_PIPELINE).  key_bytes /
 * key_offsets are device arrays under the same completeness rule as the other
 * inputs; offsets are absolute into key_bytes (m + 1 entries).  Request i's id
 * is XXH64(FormatKey(prefix, key_i), rl_cfg_seed(seed, cfg_id[i])). */
int rl_decide_batch_keys_device(rl_engine* e, size_t m, const uint8_t* key_bytes, uint64_t nbytes,
                                const uint64_t* key_offsets, uint64_t seed, const char* prefix, size_t prefix_len,
                                const int64_t* ts_ns, const int64_t* n, const uint32_t* cfg_id,
                                const int64_t* server_ms, uint8_t* decision, int64_t* remaining,
                                int64_t* retry_after_ns, int64_t* reset_at_ns, double* tokens, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* RL_KEYHASH_H */
