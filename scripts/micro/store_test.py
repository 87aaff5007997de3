"""Drive store_test.hip kernels (development microbenchmark); time with rocprofv3 --kernel-trace."""
import ctypes
import os
import sys

import torch

lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "store_test.so"))
lib.run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
n = 2048
out = torch.empty((n, n), device="cuda")
s = torch.cuda.current_stream().cuda_stream
for which, smem in [(0, 0), (1, 0), (2, 35000), (3, 35000), (2, 8192), (4, 0), (5, 35000)]:
    for _ in range(50):
        assert lib.run(which, out.data_ptr(), n, smem, s) == 0
    torch.cuda.synchronize()
print("ok")
