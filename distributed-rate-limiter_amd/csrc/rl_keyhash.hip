// On-GPU FormatKey + XXH64 of a batch of raw keys (include/rl_keyhash.h,
// SURVEY.md §8f rank 3).  Replaces the host string building of
// config.go:81-87 (FormatKey) and the Redis keyspace's string identity with a
// 64-bit id per formatted key.
//
// Layout: one workgroup hashes KH_BLOCK consecutive keys.  Their bytes are one
// contiguous range of the input buffer, so the group stages the range into LDS
// with coalesced 16-byte loads and every lane then reads its key's words from
// LDS (funnel shift of two aligned 8-byte LDS words), never from HBM with a
// stride.  A group whose range exceeds the LDS budget (keys averaging more than
// the LDS budget per key) reads its keys byte by byte from global memory.
// The host picks the group size from the mean key length nbytes / m: 256
// keys (4 waves) up to 48 B per key, else 64 keys (one wave, 192 B per key).  12 KB (not 24 KB) keeps 8 groups per CU resident: +15 % on short keys.
//
// Traffic per key: len + 8 B offset in, 8 B id out -- an HBM-bound byte kernel,
// no MFMA.
#include <hip/hip_runtime.h>

#include <cstring>
#include <string>

#include "../../include/rl_engine.h"
#include "../../include/rl_keyhash.h"

namespace {

#ifndef RL_KH_RAW_BYTES
#define RL_KH_RAW_BYTES 12288
#endif
constexpr int KH_RAW_BYTES = RL_KH_RAW_BYTES;  // staged key bytes per workgroup
constexpr int KH_RAW_WORDS = KH_RAW_BYTES / 8;
constexpr int KH_PRE_BYTES = 256;             // prefix + ':' (<= 241 bytes used)

// XXH64 constants and rounds (the published XXH64 specification, xxHash 0.8)
constexpr uint64_t P1 = 0x9E3779B185EBCA87ull;
constexpr uint64_t P2 = 0xC2B2AE3D27D4EB4Full;
constexpr uint64_t P3 = 0x165667B19E3779F9ull;
constexpr uint64_t P4 = 0x85EBCA77C2B2AE63ull;
constexpr uint64_t P5 = 0x27D4EB2F165667C5ull;

__device__ __forceinline__ uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
__device__ __forceinline__ uint64_t xround(uint64_t acc, uint64_t in) { return rotl(acc + in * P2, 31) * P1; }
__device__ __forceinline__ uint64_t xmerge(uint64_t acc, uint64_t v) { return (acc ^ xround(0, v)) * P1 + P4; }

struct Prefix {
    uint32_t len1;                 // prefix bytes + 1 for ':' (0: no prefix)
    uint8_t b[KH_PRE_BYTES];
};

// Formatted key F = prefix ':' key, read through little-endian words.  The key
// part comes from LDS (staged) or from global memory (oversized groups).
template <bool kLds>
struct Formatted {
    const uint8_t* pre;            // LDS, 8-byte aligned, zero past plen1, padded by 8
    uint32_t plen1;
    const uint64_t* raw;           // LDS words (kLds)
    uint32_t koff;                 // byte offset of the key in raw (kLds)
    const uint8_t* g;              // global key start (!kLds)

    __device__ __forceinline__ uint8_t key_byte(uint64_t j) const {
        if constexpr (kLds) return (uint8_t)(raw[(koff + j) >> 3] >> (((koff + j) & 7) * 8));
        else return g[j];
    }
    __device__ __forceinline__ uint8_t byte(uint64_t i) const {
        return i < plen1 ? pre[i] : key_byte(i - plen1);
    }
    __device__ __forceinline__ uint64_t key_word(uint64_t j) const {
        if constexpr (kLds) {
            uint64_t o = koff + j;
            uint64_t a = raw[o >> 3], b = raw[(o >> 3) + 1];
            uint32_t sh = (uint32_t)(o & 7) * 8;
            return sh ? (a >> sh) | (b << (64 - sh)) : a;
        } else {
            // byte loads (measured faster here than two aligned 8-byte loads
            // and a funnel: the lanes' keys are > 48 B apart)
            uint64_t w = 0;
            for (int k = 0; k < 8; ++k) w |= (uint64_t)g[j + k] << (8 * k);
            return w;
        }
    }
    // prefix bytes from i on; the LDS copy is zero past plen1, so a word that
    // straddles into the key has zeros in its key bytes
    __device__ __forceinline__ uint64_t pre_word(uint64_t i) const {
        const uint64_t* p64 = reinterpret_cast<const uint64_t*>(pre);
        uint64_t a = p64[i >> 3], b = p64[(i >> 3) + 1];
        uint32_t sh = (uint32_t)(i & 7) * 8;
        return sh ? (a >> sh) | (b << (64 - sh)) : a;
    }
    __device__ __forceinline__ uint64_t word(uint64_t i) const {   // bytes i..i+7, all < len
        if (i >= plen1) return key_word(i - plen1);
        uint64_t w = pre_word(i);
        const uint32_t kb = plen1 - (uint32_t)i;        // prefix bytes in this word
        if (kb < 8) {                                   // key bytes 0 .. 7-kb (< len)
            uint64_t k;
            if constexpr (kLds) {
                k = key_word(0);                        // LDS bytes past them shift out
            } else {
                k = 0;
                for (uint32_t j = 0; j < 8 - kb; ++j) k |= (uint64_t)g[j] << (8 * j);
            }
            w |= k << (8 * kb);
        }
        return w;
    }
    __device__ __forceinline__ uint32_t word32(uint64_t i) const {  // bytes i..i+3, all < len
        if (i >= plen1) {
            if constexpr (kLds) return (uint32_t)key_word(i - plen1);  // LDS reads past the key stay in the pad
        } else if (plen1 - i >= 4) {
            return (uint32_t)pre_word(i);
        }
        uint32_t w = 0;
        for (int k = 0; k < 4; ++k) w |= (uint32_t)byte(i + k) << (8 * k);
        return w;
    }
};

template <bool kLds>
__device__ uint64_t xxh64(const Formatted<kLds>& f, uint64_t len, uint64_t seed) {
    uint64_t h, p = 0;
    if (len >= 32) {
        uint64_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
        for (; p + 32 <= len; p += 32) {
            v1 = xround(v1, f.word(p));
            v2 = xround(v2, f.word(p + 8));
            v3 = xround(v3, f.word(p + 16));
            v4 = xround(v4, f.word(p + 24));
        }
        h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
        h = xmerge(h, v1);
        h = xmerge(h, v2);
        h = xmerge(h, v3);
        h = xmerge(h, v4);
    } else {
        h = seed + P5;
    }
    h += len;
    for (; p + 8 <= len; p += 8) h = rotl(h ^ xround(0, f.word(p)), 27) * P1 + P4;
    if (p + 4 <= len) {
        h = rotl(h ^ ((uint64_t)f.word32(p) * P1), 23) * P2 + P3;
        p += 4;
    }
    for (; p < len; ++p) h = rotl(h ^ ((uint64_t)f.byte(p) * P5), 11) * P1;
    h ^= h >> 33;
    h *= P2;
    h ^= h >> 29;
    h *= P3;
    h ^= h >> 32;
    return h;
}

__device__ __forceinline__ uint64_t finish_id(uint64_t h) { return h == RL_KEY_RESERVED ? RL_KEY_RESERVED - 1 : h; }

template <int KH_BLOCK>   // keys per workgroup = threads (256: 4 waves, 64: one wave)
__global__ __launch_bounds__(KH_BLOCK) void k_key_hash(const uint8_t* __restrict__ bytes, uint64_t nbytes,
                                                        const uint64_t* __restrict__ offsets, uint64_t m,
                                                        uint64_t seed, const uint32_t* __restrict__ cfg, Prefix pre,
                                                        uint64_t* __restrict__ key_id) {
    __shared__ uint64_t s_raw[KH_RAW_WORDS + 2];
    __shared__ uint64_t s_pre64[KH_PRE_BYTES / 8 + 1];
    __shared__ uint64_t s_off[KH_BLOCK + 1];

    const uint64_t b0 = (uint64_t)blockIdx.x * KH_BLOCK;
    const uint32_t nk = (uint32_t)min<uint64_t>(KH_BLOCK, m - b0);
    const uint32_t t = threadIdx.x;
    uint8_t* s_pre = reinterpret_cast<uint8_t*>(s_pre64);

    for (uint32_t i = t; i <= nk; i += KH_BLOCK) s_off[i] = offsets[b0 + i];
    for (uint32_t i = t; i < KH_PRE_BYTES; i += KH_BLOCK) s_pre[i] = pre.b[i];
    __syncthreads();

    // the group's byte range, from an aligned base; offsets out of order or past
    // nbytes make the range unusable (those keys get RL_KEY_RESERVED below)
    uint64_t lo = s_off[0], hi = s_off[nk];
    const bool range_ok = lo <= hi && hi <= nbytes;
    const uint64_t base = lo & ~(uint64_t)15;
    const uint64_t span = range_ok ? hi - base : 0;
    const bool fits = range_ok && span <= KH_RAW_BYTES;
    const bool aligned = ((uintptr_t)bytes & 15) == 0;
    if (fits) {
        const uint64_t nchunk = (span + 15) / 16;
        for (uint64_t c = t; c < nchunk; c += KH_BLOCK) {
            uint64_t g = base + c * 16;
            uint64_t w0, w1;
            if (aligned && g + 16 <= nbytes) {
                ulonglong2 v = *reinterpret_cast<const ulonglong2*>(bytes + g);   // bytes, base, g 16-aligned
                w0 = v.x;
                w1 = v.y;
            } else {                                        // the buffer's ragged tail, or an unaligned buffer
                w0 = w1 = 0;
                for (int k = 0; k < 16 && g + k < nbytes; ++k)
                    (k < 8 ? w0 : w1) |= (uint64_t)bytes[g + k] << (8 * (k & 7));
            }
            s_raw[2 * c] = w0;
            s_raw[2 * c + 1] = w1;
        }
        if (t == 0) s_raw[2 * nchunk] = s_raw[2 * nchunk + 1] = 0;   // funnel pad (never used as key bytes)
    }
    __syncthreads();
    if (t >= nk) return;

    const uint64_t a = s_off[t], z = s_off[t + 1];
    if (cfg) seed = RL_CFG_SEED(seed, cfg[b0 + t]);   // one namespace per config
    uint64_t id;
    if (!(a <= z && z <= nbytes)) {
        id = RL_KEY_RESERVED;
    } else {
        const uint64_t len = pre.len1 + (z - a);
        if (fits && a >= lo && z <= hi) {   // inside the staged range
            Formatted<true> f{s_pre, pre.len1, s_raw, (uint32_t)(a - base), nullptr};
            id = finish_id(xxh64(f, len, seed));
        } else {
            Formatted<false> f{s_pre, pre.len1, nullptr, 0, bytes + a};
            id = finish_id(xxh64(f, len, seed));
        }
    }
    key_id[b0 + t] = id;
}

int make_prefix(const char* prefix, size_t prefix_len, Prefix* out) {
    if (prefix_len > RL_KEYHASH_MAX_PREFIX || (prefix_len && !prefix)) return RL_EINVAL;
    std::memset(out, 0, sizeof *out);
    if (prefix_len) {
        std::memcpy(out->b, prefix, prefix_len);
        out->b[prefix_len] = ':';
        out->len1 = (uint32_t)prefix_len + 1;
    }
    return RL_OK;
}

}  // namespace

// The launch behind rl_hash_keys_device and the engine's raw-key path.
// mean_len: mean key length (bytes) that picks the group size -- the engine
// passes the whole batch's mean, so the chunks of a batch larger than
// max_batch choose as the batch does.  cfg (nullable): per-request config ids
// mixed into the seed (rl_cfg_seed).  The HSA grid is a 32-bit work-item count,
// so m is capped below 2^32 work-items.
int rl_hash_keys_launch(size_t m, const uint8_t* bytes, uint64_t nbytes, const uint64_t* offsets, uint64_t seed,
                        const uint32_t* cfg, const char* prefix, size_t prefix_len, double mean_len,
                        uint64_t* key_id, void* stream) {
    Prefix pre;
    if (make_prefix(prefix, prefix_len, &pre) != RL_OK) return RL_EINVAL;
    if (m == 0) return RL_OK;
    if (!offsets || !key_id || (nbytes && !bytes)) return RL_EINVAL;
    if (m > RL_KEYHASH_MAX_KEYS) return RL_EINVAL;
    // group size from the mean key length (10 % headroom: a 256-key group's
    // byte count varies little around 256 x the mean)
    const bool wide = mean_len * 1.1 > (double)KH_RAW_BYTES / 256.0 - 1.0;
    if (wide) {
        const uint64_t blocks = (m + 63) / 64;
        hipLaunchKernelGGL(k_key_hash<64>, dim3((uint32_t)blocks), dim3(64), 0, (hipStream_t)stream, bytes, nbytes,
                           offsets, (uint64_t)m, seed, cfg, pre, key_id);
    } else {
        const uint64_t blocks = (m + 255) / 256;
        hipLaunchKernelGGL(k_key_hash<256>, dim3((uint32_t)blocks), dim3(256), 0, (hipStream_t)stream, bytes, nbytes,
                           offsets, (uint64_t)m, seed, cfg, pre, key_id);
    }
    return hipGetLastError() == hipSuccess ? RL_OK : RL_EDEVICE;
}

extern "C" int rl_hash_keys_device(size_t m, const uint8_t* bytes, uint64_t nbytes, const uint64_t* offsets,
                                   uint64_t seed, const char* prefix, size_t prefix_len, uint64_t* key_id,
                                   void* stream) {
    return rl_hash_keys_launch(m, bytes, nbytes, offsets, seed, nullptr, prefix, prefix_len,
                               m ? (double)nbytes / (double)m : 0.0, key_id, stream);
}

// host XXH64 (the same specification as the device code above)
static inline uint64_t h_rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static inline uint64_t h_round(uint64_t acc, uint64_t in) { return h_rotl(acc + in * P2, 31) * P1; }
static inline uint64_t h_merge(uint64_t acc, uint64_t v) { return (acc ^ h_round(0, v)) * P1 + P4; }
static inline uint64_t h_rd64(const uint8_t* p) { uint64_t v; std::memcpy(&v, p, 8); return v; }
static inline uint32_t h_rd32(const uint8_t* p) { uint32_t v; std::memcpy(&v, p, 4); return v; }

static uint64_t xxh64_host(const uint8_t* p, uint64_t len, uint64_t seed) {
    uint64_t h, i = 0;
    if (len >= 32) {
        uint64_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
        for (; i + 32 <= len; i += 32) {
            v1 = h_round(v1, h_rd64(p + i));
            v2 = h_round(v2, h_rd64(p + i + 8));
            v3 = h_round(v3, h_rd64(p + i + 16));
            v4 = h_round(v4, h_rd64(p + i + 24));
        }
        h = h_rotl(v1, 1) + h_rotl(v2, 7) + h_rotl(v3, 12) + h_rotl(v4, 18);
        h = h_merge(h_merge(h_merge(h_merge(h, v1), v2), v3), v4);
    } else {
        h = seed + P5;
    }
    h += len;
    for (; i + 8 <= len; i += 8) h = h_rotl(h ^ h_round(0, h_rd64(p + i)), 27) * P1 + P4;
    if (i + 4 <= len) {
        h = h_rotl(h ^ ((uint64_t)h_rd32(p + i) * P1), 23) * P2 + P3;
        i += 4;
    }
    for (; i < len; ++i) h = h_rotl(h ^ ((uint64_t)p[i] * P5), 11) * P1;
    h ^= h >> 33;
    h *= P2;
    h ^= h >> 29;
    h *= P3;
    h ^= h >> 32;
    return h;
}

extern "C" int rl_hash_keys_host(size_t m, const uint8_t* bytes, uint64_t nbytes, const uint64_t* offsets,
                                 uint64_t seed, const uint32_t* cfg_id, const char* prefix, size_t prefix_len,
                                 uint64_t* key_id) {
    if (prefix_len > RL_KEYHASH_MAX_PREFIX || (prefix_len && !prefix)) return RL_EINVAL;
    if (m == 0) return RL_OK;
    if (!offsets || !key_id || (nbytes && !bytes)) return RL_EINVAL;
    for (size_t i = 0; i < m; ++i)
        if (offsets[i] > offsets[i + 1]) return RL_EINVAL;
    if (offsets[m] > nbytes) return RL_EINVAL;
    std::string buf;
    if (prefix_len) {
        buf.assign(prefix, prefix_len);
        buf.push_back(':');
    }
    const size_t plen1 = buf.size();
    for (size_t i = 0; i < m; ++i) {
        buf.resize(plen1);
        buf.append(reinterpret_cast<const char*>(bytes) + offsets[i], offsets[i + 1] - offsets[i]);
        const uint64_t sd = cfg_id ? RL_CFG_SEED(seed, cfg_id[i]) : seed;
        const uint64_t h = xxh64_host(reinterpret_cast<const uint8_t*>(buf.data()), buf.size(), sd);
        key_id[i] = h == RL_KEY_RESERVED ? RL_KEY_RESERVED - 1 : h;
    }
    return RL_OK;
}

extern "C" int rl_hash_keys(int32_t device, size_t m, const uint8_t* bytes, uint64_t nbytes, const uint64_t* offsets,
                            uint64_t seed, const char* prefix, size_t prefix_len, uint64_t* key_id) {
    Prefix pre;
    if (make_prefix(prefix, prefix_len, &pre) != RL_OK) return RL_EINVAL;
    if (m == 0) return RL_OK;
    if (!offsets || !key_id || (nbytes && !bytes)) return RL_EINVAL;
    for (size_t i = 0; i < m; ++i)
        if (offsets[i] > offsets[i + 1]) return RL_EINVAL;
    if (offsets[m] > nbytes) return RL_EINVAL;
    if (hipSetDevice(device) != hipSuccess) return RL_EDEVICE;
    uint8_t* d_bytes = nullptr;
    uint64_t *d_off = nullptr, *d_id = nullptr;
    int rc = RL_OK;
    const uint64_t nb = nbytes ? nbytes : 1;
    if (hipMalloc(&d_bytes, nb) != hipSuccess || hipMalloc(&d_off, (m + 1) * 8) != hipSuccess ||
        hipMalloc(&d_id, m * 8) != hipSuccess) {
        rc = RL_ENOMEM;
    } else if ((nbytes && hipMemcpy(d_bytes, bytes, nbytes, hipMemcpyHostToDevice) != hipSuccess) ||
               hipMemcpy(d_off, offsets, (m + 1) * 8, hipMemcpyHostToDevice) != hipSuccess) {
        rc = RL_EDEVICE;
    } else if ((rc = rl_hash_keys_device(m, d_bytes, nbytes, d_off, seed, prefix, prefix_len, d_id, nullptr)) ==
               RL_OK) {
        if (hipMemcpy(key_id, d_id, m * 8, hipMemcpyDeviceToHost) != hipSuccess) rc = RL_EDEVICE;
    }
    (void)hipFree(d_bytes);
    (void)hipFree(d_off);
    (void)hipFree(d_id);
    return rc;
}
