"""GPU: the batch collate kernels (fastspeech2/dataset.py:62-133) through
libfs2_hip.so: bit-exact against the reference collate's own output (tests/golden/
collate_ref.npz) and against the oracle at BASELINE size (B=32, T_phon<=200, T_mel<=1000)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

NAMES = ["phoneme", "speakers", "input_lengths", "mel", "pitch", "energy", "duration",
         "output_lengths", "labels", "wavs", "rank_X", "emotions"]


def _check(out, ref_get):
    for n, v in zip(NAMES, out):
        ref = ref_get(n)
        if n in ("labels", "wavs"):
            assert list(v) == [str(s) for s in list(ref)], n
        else:
            assert np.array_equal(v.cpu().numpy(), np.asarray(ref)), n


def test_gpu_collate_matches_reference_golden(cuda, golden_dir):
    import os
    from fastspeech2.dataset import GpuCollate
    from oracle.collate_oracle import items_from_golden
    z = np.load(os.path.join(golden_dir, "collate_ref.npz"))
    out = GpuCollate("cuda")(items_from_golden(z))
    assert out[3].is_contiguous() and out[3].device.type == "cuda"
    _check(out, lambda n: z["out_" + n].tolist() if n in ("labels", "wavs") else z["out_" + n])


def test_gpu_collate_full_size(cuda):
    from fastspeech2.dataset import GpuCollate
    from oracle.collate_oracle import collate_np
    g = torch.Generator().manual_seed(5)
    batch = []
    for i in range(32):
        tp = int(torch.randint(100, 201, (1,), generator=g))
        d = torch.randint(1, 10, (tp,), generator=g)
        T = int(d.sum())
        batch.append({"mel": torch.randn(80, T, generator=g), "pitch": torch.randn(T, generator=g),
                      "energy": torch.randn(T, generator=g), "duration": d,
                      "phoneme": torch.randint(1, 89, (tp,), generator=g),
                      "speaker": torch.tensor(i % 4), "emotion": torch.tensor(i % 5),
                      "text": str(i), "audio_path": f"{i}.wav"})
    out = GpuCollate("cuda")(batch)
    ref = collate_np(batch)
    _check(out, lambda n: ref[n])
