"""Generate tests/golden/keyhash_golden.json: XXH64 known answers for the
on-GPU key hashing (include/rl_keyhash.h), computed with the `xxhash` package
(python-xxhash 3.8.1 / libxxhash 0.8.2) over formatted keys
FormatKey(prefix, key) (config.go:81-87).  Run: python tests/golden/make_keyhash_golden.py
"""
import json
import os

import xxhash

cases = []
keys = [b"", b"a", b"user:123", b"192.168.0.1", b"x" * 31, b"y" * 32, b"z" * 33, bytes(range(256)),
        "tenant-é中".encode(), b"k" * 1000]
for prefix in [b"", b"ratelimit", b"api", b"p" * 240]:
    for seed in [0, 1, 7, (1 << 64) - 1]:
        for k in keys:
            f = k if not prefix else prefix + b":" + k
            cases.append({"prefix": prefix.hex(), "key": k.hex(), "seed": str(seed),
                          "xxh64": str(xxhash.xxh64_intdigest(f, seed))})
out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "keyhash_golden.json")
json.dump({"generator": "xxhash " + xxhash.VERSION + " (libxxhash " + xxhash.XXHASH_VERSION + ")",
           "cases": cases}, open(out, "w"), indent=0)
print(len(cases), "cases ->", out)
