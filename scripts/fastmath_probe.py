import ctypes, time
lib = ctypes.CDLL("tests/hip/build/libsf_fastmath_check.so")
c = (ctypes.c_ulonglong * 6)()
t = time.time(); rc = lib.sf_fastmath_check(c); print("rc", rc, "s", round(time.time() - t, 3), list(c))
