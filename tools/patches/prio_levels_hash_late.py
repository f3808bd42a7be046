# A/B: later priority steps (12/14/15 sixteenths) for hash workgroups with >= 64 items only (one
# GPU); dense and small hash shares keep 8/13/15.
import sys

p = sys.argv[1]
s = open(p).read()
old = "const int p = q < mine * 8u ? 3 : q < mine * 13u ? 2 : q < mine * 15u ? 1 : 0;"
assert old in s
new = ("const bool late = HASH && mine >= 64u;\n"
       "                const int p = q < mine * (late ? 12u : 8u) ? 3 : q < mine * (late ? 14u : 13u) ? 2 "
       ": q < mine * 15u ? 1 : 0;")
s = s.replace(old, new)
open(p, "w").write(s)
