"""Times pv_decoder_tail_f16 alone at configs[2]'s shape (batch 32, fm
240 x 320 x 32 -> out 480 x 640 x 20), eager launches between events.
    PVVOTE_LIB=variants/x.so python tools/tail_probe.py [iters]"""
import sys
import torch
sys.path.insert(0, ".")
from pvnet_amd.network import decoder_tail, decoder_tail_weights  # noqa: E402

it = int(sys.argv[1]) if len(sys.argv) > 1 else 20
cl = torch.channels_last
torch.manual_seed(0)
n, h, w = 32, 240, 320
fm = torch.randn(n, 32, h, w, device="cuda").half().contiguous(memory_format=cl)
img = torch.randn(n, 3, 2 * h, 2 * w, device="cuda").half().contiguous(memory_format=cl)
c0 = torch.nn.Conv2d(35, 32, 3, 1, 1).cuda().half()
c1 = torch.nn.Conv2d(32, 20, 1).cuda().half()
wts = decoder_tail_weights(c0, c1)
for _ in range(3):
    decoder_tail(fm, img, wts)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(it):
    decoder_tail(fm, img, wts)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 1e3 / it
px = n * 4 * h * w
print(f"decoder_tail: {us:.1f} us/launch  {px / us / 1e3:.2f} Gpx/s  "
      f"{(fm.numel() * 2 + img.numel() * 2 + px * 40) / us / 1e6:.2f} TB/s algorithmic")
