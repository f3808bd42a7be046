# Diagnostic: per-item durations of the hash z-half protocol's categories in the TSDF_HASH_DIAG
# counters (tools/gpu/hash_diag.py).  Applies hash_item_times.diff to the copy of csrc/:
#   tools/build_patched.sh hdiag tools/patches/hash_item_times.py "-DTSDF_HASH_DIAG"
import os
import subprocess
import sys

csrc = os.path.dirname(os.path.abspath(sys.argv[1]))
diff = os.path.join(os.path.dirname(os.path.abspath(__file__)), "hash_item_times.diff")
subprocess.run(["patch", "-s", "-d", csrc, "-p3", "-i", diff], check=True)
