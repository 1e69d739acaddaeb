import torch
a = torch.empty((2160, 3840, 4), dtype=torch.uint8, device="cuda")
b = torch.empty_like(a)
for _ in range(50):
    b.copy_(a)
torch.cuda.synchronize()
