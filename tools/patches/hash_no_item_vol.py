# A/B: the hash integrate reads the volume once per launch (no per-item opaque re-read)
import sys
p = sys.argv[1]
s = open(p).read()
old = "__device__ inline const Vol& item_vol(const Vol& v) { return *(const Vol*)opaque((VolP)&v); }"
assert old in s
s = s.replace(old, "__device__ inline const Vol& item_vol(const Vol& v) { return v; }")
open(p, "w").write(s)
