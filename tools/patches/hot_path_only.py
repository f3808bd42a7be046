import sys
p=sys.argv[1]; s=open(p).read()
# hot path only: no slow projection fix-up, fast colour path always, LDS table always
s=s.replace("if (__ballot(any_slow)) {", "if (false) {")
s=s.replace("        if (fast_c) {\n            // Steps in pairs", "        if (true) {\n            // Steps in pairs")
s=s.replace("                if (fast_t) {\n                    y[0] = *(const double*)((const char*)s_rcp + o0);", "                if (true) {\n                    y[0] = *(const double*)((const char*)s_rcp + o0);")
open(p,'w').write(s)
