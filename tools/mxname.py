import sys, torch
sys.path[:0] = ["/root/repo", "/root/repo/aa-clip_amd"]
from aaclip import ops, _lib
dev = torch.device("cuda:0")
FP8 = torch.float8_e4m3fn
M, N, K = 4096, 1024, 1024
a = torch.randn(M, K, device=dev)
a8 = torch.empty(M, K, device=dev, dtype=FP8); asc = ops.mx_scales(M, K, dev); ops.quant_fp8_mx(a, a8, asc)
w8 = torch.randn(N, K, device=dev).to(FP8); sw = torch.ones(N, device=dev)
out = torch.empty(M, N, device=dev)
for v in (0, 6, 0):
    _lib.call("aaclip_set_gemm_variant", v)
    for _ in range(3): ops.gemm_fp8mx(a8, asc, w8, sw, out)
    torch.cuda.synchronize()
print("done")
