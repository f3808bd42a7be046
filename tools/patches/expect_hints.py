import sys
p=sys.argv[1]; s=open(p).read()
for a,b in [("    if (__ballot(any_slow)) {", "    if (__builtin_expect(__ballot(any_slow) != 0, 0)) {"),
            ("        if (__ballot(any_ld)) {", "        if (__builtin_expect(__ballot(any_ld) != 0, 0)) {"),
            ("        if (fast_c) {", "        if (__builtin_expect(fast_c, 1)) {"),
            ("                if (fast_t) {", "                if (__builtin_expect(fast_t, 1)) {")]:
    assert a in s, a
    s=s.replace(a,b)
open(p,'w').write(s)
