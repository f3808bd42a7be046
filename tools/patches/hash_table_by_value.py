# A/B: the fused hash launch reads its table from the by-value argument (no opaque pointer)
import sys
p = sys.argv[1]
s = open(p).read()
old = "    const Table& tab = *(const Table*)opaque(&A->tab);"
assert old in s
s = s.replace(old, "    const Table& tab = a.tab;")
open(p, "w").write(s)
