import sys; sys.path.insert(0, '/root/repo/aa-clip_amd'); sys.path.insert(0, '/root/repo')
import torch
from aaclip import ops
dev = torch.device('cuda:0'); FP8 = torch.float8_e4m3fn
M, N, K = 256, 256, 256
a = torch.ones(M, K, device=dev).to(FP8)
w = torch.zeros(N, K, device=dev)
for n in range(N): w[n, (n * 5) % K] = 1.0  # output n picks k = 5n mod K
w8 = w.to(FP8); sw = torch.ones(N, device=dev)
sc = torch.full((K // 128, M, 2), 127, device=dev, dtype=torch.uint8)
out = torch.empty(M, N, device=dev)
ops.gemm_fp8mx(a, sc, w8, sw, out); torch.cuda.synchronize()
print('unit scales: unique', out.unique().tolist()[:10])
# set the scale of row 3, block 1 (k 64..127) to 2^3
sc[0, 3, 1] = 130
ops.gemm_fp8mx(a, sc, w8, sw, out); torch.cuda.synchronize()
changed = (out != 1).nonzero().tolist()
print('changed count', len(changed), changed[:12])
ks = sorted(set((c[1] * 5) % K for c in changed))
print('k of changed cols', ks[:20], '... rows', sorted(set(c[0] for c in changed))[:20])
