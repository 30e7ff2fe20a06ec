import torch, time
print("preferred blas:", torch.backends.cuda.preferred_blas_library())
for (m, k, n) in [(64, 64, 64), (2500, 64, 128), (25000, 128, 64), (2500, 1088, 64), (32, 50, 50)]:
    a = torch.randn(m, k, device="cuda"); w = torch.randn(n, k, device="cuda", requires_grad=True)
    y = torch.nn.functional.linear(a, w); y.sum().backward(); torch.cuda.synchronize()
    print("ok", m, k, n, float(y.abs().mean()))
