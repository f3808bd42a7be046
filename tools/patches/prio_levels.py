# A/B: the progress priority's steps (in 16ths of a workgroup's share taken: priority 3 below the
# first, 2 below the second, 1 below the third, then 0).  PRIO_LEVELS="a,b,c" in the environment.
import os
import sys

p = sys.argv[1]
s = open(p).read()
old = "const int p = q < mine * 8u ? 3 : q < mine * 13u ? 2 : q < mine * 15u ? 1 : 0;"
assert old in s
a, b, c = os.environ["PRIO_LEVELS"].split(",")
s = s.replace(old, f"const int p = q < mine * {a}u ? 3 : q < mine * {b}u ? 2 : q < mine * {c}u ? 1 : 0;")
open(p, "w").write(s)
