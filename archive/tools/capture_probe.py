"""What hipStreamIsCapturing reports for the null stream, a torch stream, and a stream
inside torch.cuda.graph capture (tools probe, not product)."""
import ctypes

import torch

torch.cuda.set_device(0)
torch.empty(1, device="cuda")
hip = ctypes.CDLL("libamdhip64.so")
st = ctypes.c_int(-1)


def q(s):
    st.value = -1
    rc = hip.hipStreamIsCapturing(ctypes.c_void_p(s), ctypes.byref(st))
    return rc, st.value


print("null stream:", q(0))
s = torch.cuda.Stream()
print("torch stream:", q(s.cuda_stream))
print("current stream:", q(torch.cuda.current_stream().cuda_stream))
g = torch.cuda.CUDAGraph()
x = torch.zeros(4, device="cuda")
with torch.cuda.graph(g):
    print("capturing stream:", q(torch.cuda.current_stream().cuda_stream))
    x += 1
print("after capture, null:", q(0))
