"""Stand-in for numba, used ONLY by tools/gen_golden.py to import the reference in this container.

numba is not installed here.  `njit` becomes an identity decorator and `prange` becomes `range`.
The numerically relevant helpers are then replaced by numba-typing-faithful NumPy versions
(tools/gen_golden.py: `faithful_patch`), so the reference's CPU integrate() runs with the same
arithmetic numba would have compiled.  Never imported by the product or the tests.
"""


def njit(*args, **kwargs):
    if len(args) == 1 and callable(args[0]) and not kwargs:
        return args[0]
    return lambda f: f


jit = njit
prange = range
