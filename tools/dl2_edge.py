"""Long-token decrypt at small token counts (edge probe): python tools/dl2_edge.py N [L]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import reticulum_amd as rt
    from reticulum_amd import device
    n = int(sys.argv[1])
    L = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    tl = rt.token_len(L)
    g = torch.Generator(device="cuda").manual_seed(n)
    pt = torch.randint(0, 256, (n, L), dtype=torch.uint8, device="cuda", generator=g)
    iv = torch.randint(0, 256, (n, 16), dtype=torch.uint8, device="cuda", generator=g)
    ks = rt.KeySet(bytes(range(64)))
    tok = torch.empty((n, tl), dtype=torch.uint8, device="cuda")
    device.encrypt_uniform(ks, pt, L, iv, tok)
    torch.cuda.synchronize()
    print("encrypt ok", flush=True)
    back = torch.empty((n, tl - 48), dtype=torch.uint8, device="cuda")
    ol = torch.empty(n, dtype=torch.int32, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    device.decrypt_uniform(ks, tok, tl, back, ol, st)
    torch.cuda.synchronize()
    print("decrypt", n, L, "ok" if int(st.abs().sum()) == 0 and torch.equal(back[:, :L], pt) else "MISMATCH", flush=True)


if __name__ == "__main__":
    main()
