"""MI355X-native FastSpeech2-with-emotion-intensity train path (drop-in for
Orca0917/fine-grained-emotional-control-of-tts ``emo_rank_tts/fastspeech2``).

    from fastspeech2.model import FastSpeech2      # model.py:32  (same kwargs, 8-tuple)
    from fastspeech2.loss import Loss              # loss.py:6    (same dict of 7 losses)
    from fastspeech2.train import train_step, FusedTrainer
    from fastspeech2.optim import FusedAdamW

Compute runs only through libfs2_hip.so (include/fs2_hip.h); see DESIGN.md.
"""

import os

import yaml

_HERE = os.path.dirname(os.path.abspath(__file__))


def load_config(path=None):
    """parameter.yaml with the reference's key names (fastspeech2/parameter.yaml)."""
    with open(path or os.path.join(_HERE, "parameter.yaml")) as f:
        return yaml.safe_load(f)
