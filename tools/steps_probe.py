import sys, time, torch
sys.path.insert(0, '/root/repo')
import reticulum_amd as rt
from reticulum_amd import device
n, L = 1 << 20, 500
tl = rt.token_len(L)
g = torch.Generator(device='cuda').manual_seed(1)
pt = torch.randint(0, 256, (n, L), dtype=torch.uint8, device='cuda', generator=g)
iv = torch.randint(0, 256, (n, 16), dtype=torch.uint8, device='cuda', generator=g)
tok = torch.empty((n, tl), dtype=torch.uint8, device='cuda')
back = torch.empty((n, tl - 48), dtype=torch.uint8, device='cuda')
ol = torch.empty(n, dtype=torch.int32, device='cuda'); st = torch.empty(n, dtype=torch.int32, device='cuda')
import numpy as np
ks = rt.KeySet(np.arange(64, dtype=np.uint8).reshape(1, 64), device=0)
s = torch.cuda.current_stream()
def step(ev):
    ev[0].record(s); device.encrypt_uniform(ks, pt, L, iv, tok, stream=s); ev[1].record(s)
    device.decrypt_uniform(ks, tok, tl, back, ol, st, stream=s); ev[2].record(s)
for mode in ('after_idle', 'continuous'):
    for _ in range(3): step([torch.cuda.Event(enable_timing=True) for _ in range(3)])
    torch.cuda.synchronize()
    if mode == 'after_idle':
        time.sleep(0.05)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(40)]
    for e in evs: step(e)
    torch.cuda.synchronize()
    print(mode, ' '.join('%.3f' % (e[0].elapsed_time(e[1]) + e[1].elapsed_time(e[2])) for e in evs))
