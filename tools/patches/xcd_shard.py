"""Timing experiment (A/B): record shards partitioned by XCD (workgroup i runs on XCD i % 8),
so a shard counter's atomics come from one XCD only."""
import sys
p = sys.argv[1] + "/pm_kernels.h"
s = open(p).read()
o = "__device__ __forceinline__ uint32_t shard_of(uint32_t salt, int tile) { return (salt * 31u + (uint32_t)tile * 7919u) % kShards; }"
assert o in s
s = s.replace(o, "__device__ __forceinline__ uint32_t shard_of(uint32_t salt, int tile) { return (blockIdx.x & 7u) * (kShards / 8) + (salt * 31u + (uint32_t)tile * 7919u) % (kShards / 8); }")
open(p, "w").write(s)
