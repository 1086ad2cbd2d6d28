"""LayerNorm kernels at the bench's decoder / encoder shapes, as FS2Engine._fft_fwd/_fft_bwd
issue them (bf16, dropout 0.1 on the residual branch, gamma/beta/column-sum partials):
us per call and GB/s of algorithmic traffic."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fine-grained-emotional-control-of-tts_amd"))
import torch  # noqa: E402


def timed(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


def main():
    from fastspeech2 import ops, _native
    _native.load()
    D = 384
    bf = torch.bfloat16
    for M in (31264, 6400):
        r = lambda: (torch.randn(M, D, device="cuda") * 0.5).to(bf)
        X, R, dY = r(), r(), r()
        g, be = torch.rand(D, device="cuda") + 0.5, torch.randn(D, device="cuda") * 0.1
        Y, S = torch.empty_like(X), torch.empty_like(X)
        mean = torch.empty(M, device="cuda")
        rstd = torch.empty_like(mean)
        fwd = lambda: ops.ln_fwd(X, D, g, be, 1e-6, Y, D, mean, rstd, M, D, dt=1, seed=7, r=R, ldr=D,
                                 p_r=0.1, salt_r=3, s_out=S)
        us = timed(fwd)
        print(f"M={M} ln_fwd  {us:7.1f} us  {4 * M * D * 2 / us / 1e3:7.0f} GB/s", flush=True)
        dS, dR = torch.empty_like(X), torch.empty_like(X)
        dg, db, dc = (torch.zeros(D, device="cuda") for _ in range(3))
        ws = torch.empty(int(ops.ln_ws(M, D)), device="cuda")
        bwd = lambda: ops.ln_bwd(dY, D, S, D, mean, rstd, g, be, dS, D, M, D, dt=1, ws=ws, seed=7,
                                 dr=dR, p_r=0.1, salt_r=3, dgamma=dg, dbeta=db, dcol=dc)
        us = timed(bwd)
        print(f"M={M} ln_bwd  {us:7.1f} us  {4 * M * D * 2 / us / 1e3:7.0f} GB/s", flush=True)
        if os.environ.get("LN_VARIANTS"):
            v = {
                "no dropout": lambda: ops.ln_bwd(dY, D, S, D, mean, rstd, g, be, dS, D, M, D, dt=1,
                                                 ws=ws, seed=7, dr=dR, p_r=0.0, salt_r=3, dgamma=dg,
                                                 dbeta=db, dcol=dc),
                "no partials": lambda: ops.ln_bwd(dY, D, S, D, mean, rstd, g, be, dS, D, M, D, dt=1,
                                                  ws=ws, seed=7, dr=dR, p_r=0.1, salt_r=3),
                "no dr": lambda: ops.ln_bwd(dY, D, S, D, mean, rstd, g, be, dS, D, M, D, dt=1, ws=ws,
                                            seed=7),
            }
            for name, fn in v.items():
                us = timed(fn)
                print(f"M={M} ln_bwd {name:12s} {us:7.1f} us", flush=True)
            for name, fn in {"copy": lambda: dS.copy_(dY), "add": lambda: torch.add(dY, S, out=dS)}.items():
                us = timed(fn)
                print(f"M={M} torch {name:12s} {us:7.1f} us", flush=True)


def postnet_case():
    """PostNet LayerNorm backward: D = 512, tanh gate, output dropout, gamma / beta / bias
    partials, no residual-branch output (engine._postnet_bwd)."""
    from fastspeech2 import ops
    M, D = 31264, 512
    bf = torch.bfloat16
    X = (torch.randn(M, D, device="cuda") * 0.5).to(bf)
    dY = (torch.randn(M, D, device="cuda") * 0.5).to(bf)
    g, be = torch.rand(D, device="cuda") + 0.5, torch.randn(D, device="cuda") * 0.1
    Y = torch.empty_like(X)
    mean = torch.empty(M, device="cuda")
    rstd = torch.empty_like(mean)
    ops.ln_fwd(X, D, g, be, 1e-5, Y, D, mean, rstd, M, D, dt=1, seed=7, do_tanh=1, p_o=0.5,
               salt_o=5)
    dS = torch.empty_like(X)
    dg, db, dc = (torch.zeros(D, device="cuda") for _ in range(3))
    ws = torch.empty(int(ops.ln_ws(M, D)), device="cuda")
    bwd = lambda: ops.ln_bwd(dY, D, X, D, mean, rstd, g, be, dS, D, M, D, dt=1, ws=ws, seed=7,
                             do_tanh=1, p_o=0.5, salt_o=5, dgamma=dg, dbeta=db, dcol=dc)
    us = timed(bwd)
    print(f"M={M} D=512 tanh ln_bwd {us:7.1f} us  {4 * M * D * 2 / us / 1e3:7.0f} GB/s", flush=True)
    fwd = lambda: ops.ln_fwd(X, D, g, be, 1e-5, Y, D, mean, rstd, M, D, dt=1, seed=7, do_tanh=1,
                             p_o=0.5, salt_o=5)
    us = timed(fwd)
    print(f"M={M} D=512 tanh ln_fwd {us:7.1f} us", flush=True)


if __name__ == "__main__":
    if os.environ.get("LN_POSTNET"):
        from fastspeech2 import _native
        _native.load()
        postnet_case()
        sys.exit(0)
    main()
