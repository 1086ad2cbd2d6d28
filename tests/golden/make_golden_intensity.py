"""Generates tests/golden/intensity_ref.npz from the REFERENCE itself (run in the dev container,
where /root/reference exists; the GPU box never runs this).

    python tests/golden/make_golden_intensity.py

* ``IntensityExtractor`` comes from /root/reference/emo_rank_tts/rank_model/model.py by an
  ordinary import (it needs only torch).
* ``get_intensity_representation`` lives in fastspeech2/train.py, whose module imports
  speechbrain / tensorboard (absent here).  The function itself uses only torch, so this script
  reads train.py as text, compiles that ONE function definition (ast) and calls it -- the
  reference's own code on our inputs, no stand-in modules.  Its ``rank_X`` is given in the
  (B, T, n_mels+2) layout the extractor actually reads (the collate's
  (B, n_mels+2, T) tensor would raise inside the reference).

Fixture (small config so it stays ~100 KB): n_mels=14 (C=16), 2 heads, 5 emotions, 2 layers,
hidden 32, kernel 9, eval mode; B=3, T=40, lengths [40, 31, 17]; ragged phoneme durations with a
zero-duration phoneme.  Stored: the extractor state_dict, inputs, I = extractor(x) and the
phoneme-level representation.
"""
import ast
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/emo_rank_tts"

CFG = dict(n_mels=14, n_heads=2, n_emotions=5, n_encoder_layers=2, hidden_dim=32, kernel_size=9,
           dropout=0.1)


def _reference_function(path, name):
    src = open(path).read()
    tree = ast.parse(src)
    fn = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == name]
    assert len(fn) == 1, name
    mod = ast.Module(body=fn, type_ignores=[])
    ns = {"torch": torch}
    exec(compile(mod, path, "exec"), ns)
    return ns[name]


def main():
    sys.path.insert(0, REF)
    from rank_model.model import IntensityExtractor  # reference module (torch only)
    get_rep = _reference_function(os.path.join(REF, "fastspeech2", "train.py"),
                                  "get_intensity_representation")
    torch.manual_seed(11)
    ext = IntensityExtractor(**CFG).eval().requires_grad_(False)
    B, T, C = 3, 40, CFG["n_mels"] + 2
    lengths = torch.tensor([40, 31, 17])
    x = torch.randn(B, T, C)
    for b in range(B):
        x[b, int(lengths[b]):] = 0.0                    # collate zero padding
    emotions = torch.tensor([3, 0, 4])
    # phoneme durations summing to each mel length (one zero-duration phoneme)
    durs = [[3, 5, 0, 7, 2, 6, 4, 9, 4], [6, 2, 8, 5, 4, 6], [5, 1, 7, 4]]
    Tp = max(len(d) for d in durs)
    duration = torch.zeros(B, Tp, dtype=torch.long)
    for b, d in enumerate(durs):
        assert sum(d) == int(lengths[b])
        duration[b, :len(d)] = torch.tensor(d)
    phon_len = torch.tensor([len(d) for d in durs])
    phoneme = (duration > 0).long() + 1
    with torch.no_grad():
        I = ext(x, lengths, emotions)
    batch = (phoneme, None, phon_len, None, None, None, duration, lengths, None, None, x,
             emotions)
    rep = get_rep(ext, batch, torch.device("cpu"))
    sd = {k: v.numpy() for k, v in ext.state_dict().items()}
    np.savez_compressed(os.path.join(HERE, "intensity_ref.npz"), x=x.numpy(),
                        lengths=lengths.numpy(), emotions=emotions.numpy(),
                        duration=duration.numpy(), phon_len=phon_len.numpy(), I=I.numpy(),
                        rep=rep.numpy(), cfg_keys=np.array(list(CFG)),
                        cfg_vals=np.array([float(v) for v in CFG.values()]),
                        **{"sd." + k: v for k, v in sd.items()})
    print("wrote intensity_ref.npz", I.shape, rep.shape)


if __name__ == "__main__":
    main()
