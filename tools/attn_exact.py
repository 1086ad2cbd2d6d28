"""Bit-exactness of the fused attention backward variants of the experiments library
(FS2_ATTN_BWD bits) against the default kernels, at the bench's decoder / encoder shapes."""
import math
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fine-grained-emotional-control-of-tts_amd"))
import torch  # noqa: E402


def main():
    from fastspeech2 import ops, _native
    _native.load()
    B, H, dh = 32, 2, 192
    D = H * dh
    var = os.environ.get("ATTN_VARIANT", "4")
    ok = True
    for T in (977, 200):
        g = torch.Generator().manual_seed(T)
        lens = sorted([T] + torch.randint(T // 2, T + 1, (B - 1,), generator=g).tolist(), reverse=True)
        qkv = (torch.randn(B * T, 3 * D, device="cuda") * 0.5).to(torch.bfloat16)
        kp = torch.zeros(B, T, dtype=torch.uint8, device="cuda")
        for b, L in enumerate(lens):
            kp[b, L:] = 1
        out = torch.empty(B * T, D, device="cuda", dtype=torch.bfloat16)
        lse = torch.empty(B * H, T, device="cuda")
        dout = torch.randn(B * T, D, device="cuda").to(torch.bfloat16)
        ws = torch.empty(int(ops.attn_ws(B, H, T)), device="cuda")
        sc = 1.0 / math.sqrt(dh)
        for p in (0.0, 0.1):
            ops.attn_fwd(qkv, 3 * D, kp, B, H, T, dh, sc, p, 1, 2, out, D, lse, dt=1)
            res = []
            for v in ("0", var):
                os.environ["FS2_ATTN_BWD"] = v
                dqkv = torch.full((B * T, 3 * D), float("nan"), device="cuda", dtype=torch.bfloat16)
                ops.attn_bwd(qkv, 3 * D, kp, out, D, dout, D, lse, B, H, T, dh, sc, p, 1, 2,
                             dqkv, 3 * D, dt=1, ws=ws)
                torch.cuda.synchronize()
                res.append(dqkv)
            for i, nm in enumerate("QKV"):
                a, b = res[0][:, i * D:(i + 1) * D].float(), res[1][:, i * D:(i + 1) * D].float()
                nan = torch.isnan(b).sum().item()
                same = torch.equal(a, b)
                rel = ((a - b).abs().max() / a.abs().max()).item()
                print(f"T={T} p={p} d{nm}: bit-identical={same} max rel diff {rel:.2e} nan {nan}", flush=True)
                if not same and os.environ.get("ATTN_DIAG"):
                    bad = (a != b) & ~(torch.isnan(a) & torch.isnan(b))
                    r, c = bad.nonzero(as_tuple=True)
                    bb, tt = r // T, r % T
                    print("  rows with diffs:", r.unique().numel(), "of", B * T, " batches:",
                          bb.unique().tolist()[:40], flush=True)
                    print("  key idx mod 128 hist:", torch.bincount(tt % 128, minlength=128).tolist(), flush=True)
                    print("  key block hist:", torch.bincount(tt // 128).tolist(), flush=True)
                    print("  col hist (per 16):", torch.bincount(c // 16).tolist(), flush=True)
                    print("  nan in ref:", torch.isnan(a).sum().item(), flush=True)
                ok = ok and same
    os.environ["FS2_ATTN_BWD"] = "0"
    print("ALL BIT-IDENTICAL" if ok else "DIFFERENCES", flush=True)


if __name__ == "__main__":
    main()
