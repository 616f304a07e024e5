"""Known-bytes read for FETCH_SIZE calibration: sums a 4 GiB int32 tensor
(torch reduction: 16-B vector loads) a few times."""
import torch

x = torch.ones(1 << 30, dtype=torch.int32, device="cuda")   # 4 GiB
for _ in range(3):
    s = x.sum()
torch.cuda.synchronize()
print(int(s))
