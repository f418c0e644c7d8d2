import torch
bf = torch.bfloat16
for M, N, K in [(65536, 3072, 1024), (65536, 17920, 4096), (65536, 1024, 4096)]:
    x = torch.rand(M, K, device="cuda").to(bf)
    w = torch.rand(N, K, device="cuda").to(bf)
    for _ in range(3):
        y = torch.matmul(x, w.t())
torch.cuda.synchronize()
