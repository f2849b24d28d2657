"""Which HIP flags do torch's pool streams carry (blocking = 0, non-blocking = 1)?"""
import ctypes

import torch

hip = ctypes.CDLL("libamdhip64.so")
s = torch.cuda.Stream()
flags = ctypes.c_uint(99)
rc = hip.hipStreamGetFlags(ctypes.c_void_p(s.cuda_stream), ctypes.byref(flags))
print("pool stream flags", rc, flags.value)
d = torch.cuda.current_stream()
rc = hip.hipStreamGetFlags(ctypes.c_void_p(d.cuda_stream), ctypes.byref(flags))
print("current stream", d.cuda_stream, "flags", rc, flags.value)
