"""Inference throughput (BASELINE config 5): 256 sentences with random speaker /
emotion / intensity level from a synthetic prototype bank, mel generation with predicted
durations in ONE bf16 batch on 1 MI355X (vocoder out of scope).  Random-init weights; the
duration predictor's output bias is set to log(1 + 5) so sentences get ~5 frames per phoneme.

    python tools/infer_bench.py [--sentences 256] [--steps 10] [--warmup 3]
Prints one JSON line: mel-frames/s (forward only) and the achieved forward TFLOP/s.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fine-grained-emotional-control-of-tts_amd"))

import numpy as np
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sentences", type=int, default=256)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--vocoder", action="store_true",
                    help="also decode the mels with the HiFi-GAN generator (fastspeech2.vocoder)")
    a = ap.parse_args()
    from fastspeech2 import load_config
    from fastspeech2.model import FastSpeech2
    from fastspeech2.inference import get_intensity_rep, synthesize
    from fastspeech2.flops import forward_flops
    cfg = load_config()
    torch.manual_seed(0)
    m = FastSpeech2(**cfg["model"]["fastspeech2"], n_speakers=4,
                    act_dtype=torch.bfloat16).cuda().eval()
    with torch.no_grad():
        m.durPred.linear.w.weight.mul_(0.05)
        m.durPred.linear.w.bias.fill_(float(np.log1p(5.0)))
    g = torch.Generator().manual_seed(1)
    bank = np.random.default_rng(2).standard_normal((4, 5, 3, 5)).astype(np.float32)
    phs, spk, inten = [], [], []
    for i in range(a.sentences):
        n = int(torch.randint(30, 81, (1,), generator=g))
        phs.append(torch.randint(1, 95, (n,), generator=g))
        s, e, lv = i % 4, (i // 4) % 5, (i // 20) % 3
        spk.append(s)
        inten.append(get_intensity_rep(s, e, lv, n, bank)[0])
    for _ in range(a.warmup):
        mels, lens = synthesize(m, phs, spk, inten)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        mels, lens = synthesize(m, phs, spk, inten)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    frames = sum(lens)
    Tp, Tm = max(p.numel() for p in phs), max(lens)
    fl = forward_flops(m.cfg, a.sentences, Tp, Tm)
    voc = None
    if a.vocoder:
        from fastspeech2.vocoder import HifiganGenerator
        from fastspeech2.flops import vocoder_flops
        gen = HifiganGenerator(act_dtype=torch.bfloat16).cuda()
        # mels padded to T_mel_max as (B, 80, T) (decode_batch's input layout)
        melb = torch.zeros(a.sentences, 80, Tm, device="cuda")
        for i, x in enumerate(mels):
            melb[i, :, :x.shape[0]] = x.float().t()
        wav = gen.decode_batch(melb)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            wav = gen.decode_batch(melb)
        torch.cuda.synchronize()
        tv = (time.perf_counter() - t0) / a.steps
        vf = vocoder_flops(a.sentences, Tm)
        voc = {"ms_per_batch": tv * 1e3, "samples_per_s": wav.numel() / tv,
               "padded_samples": wav.numel(), "tflops_padded": vf / tv / 1e12,
               "end_to_end_mel_frames_per_s": frames / (dt + tv),
               "note": "HiFi-GAN generator (LibriTTS-16k architecture), random weights, bf16"}
    print(json.dumps({"metric": "inference mel-frames/sec (mel generation, predicted durations)",
                      "value": frames / dt, "unit": "mel-frames/s", "ms_per_batch": dt * 1e3,
                      "sentences": a.sentences, "T_phon_max": Tp, "T_mel_max": Tm,
                      "frames": frames, "dtype": "bf16", "tflops_padded": fl / dt / 1e12,
                      "note": "includes host padding of the sentence list and the mel-length "
                              "D2H the reference also performs (mel_lens on CPU)",
                      "vocoder": voc}))


if __name__ == "__main__":
    main()
