"""Generates tests/golden/collate_ref.npz from the REFERENCE collate (dev container only).

    python tests/golden/make_golden_collate.py

``TextMelCollateWithAlignment`` lives in fastspeech2/dataset.py, whose module imports
fastspeech2/util.py (speechbrain, absent here).  The class itself uses only torch, so this
script compiles that ONE class definition from the file (ast) and calls it on seeded items in
the dataset's item layout (dataset.py:46-58): the reference's own code, no stand-in modules.
Items include equal phoneme lengths, so the fixture also pins the order ``torch.sort`` gives
ties.
"""
import ast
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/emo_rank_tts/fastspeech2/dataset.py"


def _reference_class(path, name):
    tree = ast.parse(open(path).read())
    cls = [n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == name]
    assert len(cls) == 1, name
    ns = {"torch": torch}
    exec(compile(ast.Module(body=cls, type_ignores=[]), path, "exec"), ns)
    return ns[name]


def items(seed=0, n_mels=80):
    g = torch.Generator().manual_seed(seed)
    tps = [13, 21, 13, 8, 21, 17]          # ties on purpose
    out = []
    for i, tp in enumerate(tps):
        d = torch.randint(0, 7, (tp,), generator=g)
        T = int(d.sum())
        out.append({"mel": torch.randn(n_mels, T, generator=g),
                    "pitch": torch.randn(T, generator=g), "energy": torch.randn(T, generator=g),
                    "duration": d, "phoneme": torch.randint(1, 89, (tp,), generator=g),
                    "speaker": torch.tensor(i % 4), "emotion": torch.tensor((3 * i) % 5),
                    "text": f"utt {i}", "audio_path": f"/wav/{i}.wav"})
    return out


def main():
    collate = _reference_class(REF, "TextMelCollateWithAlignment")()
    its = items()
    out = collate(its)
    names = ["phoneme", "speakers", "input_lengths", "mel", "pitch", "energy", "duration",
             "output_lengths", "labels", "wavs", "rank_X", "emotions"]
    arrs = {}
    for n, v in zip(names, out):
        if isinstance(v, torch.Tensor):
            arrs["out_" + n] = v.contiguous().numpy()
        else:
            arrs["out_" + n] = np.array(v)
    for i, it in enumerate(its):
        for k in ("mel", "pitch", "energy", "duration", "phoneme", "speaker", "emotion"):
            arrs[f"in{i}_{k}"] = it[k].numpy()
        arrs[f"in{i}_text"] = np.array(it["text"])
        arrs[f"in{i}_audio_path"] = np.array(it["audio_path"])
    arrs["n_items"] = np.array(len(its))
    np.savez_compressed(os.path.join(HERE, "collate_ref.npz"), **arrs)
    print("wrote collate_ref.npz", {k: v.shape for k, v in arrs.items() if k.startswith("out_")})


if __name__ == "__main__":
    main()
