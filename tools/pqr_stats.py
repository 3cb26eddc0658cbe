import os, sys, torch
sys.path.insert(0, "/root/repo")
import gptq_svd_amd.gptq_utils as g
dev = torch.device("cuda")
torch.manual_seed(1)
n = int(os.environ.get("N", "4096"))
acc = g.HessianAccumulator(n, dev)
acc.add_batch(torch.randn(3 * n // 4, n, device=dev).half())
H = acc.get_hessian()
for _ in range(3):
    g.process_hessian_alt(H, 1e-4, "energy")
torch.cuda.synchronize()
print("done")
