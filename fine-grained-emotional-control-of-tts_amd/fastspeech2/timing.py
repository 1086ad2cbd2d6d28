"""HIP-event timing of tagged kernel launches on the launching (current) stream."""

import torch


class KernelTimer:
    def __init__(self):
        self.pending = {}
        self.pairs = {}

    def start(self, tag):
        e = torch.cuda.Event(enable_timing=True)
        e.record(torch.cuda.current_stream())
        self.pending[tag] = e

    def stop(self, tag):
        e = torch.cuda.Event(enable_timing=True)
        e.record(torch.cuda.current_stream())
        self.pairs.setdefault(tag, []).append((self.pending.pop(tag), e))

    def reset(self):
        self.pending, self.pairs = {}, {}

    def summary(self):
        """tag -> (launches, mean ms); call after a synchronize."""
        out = {}
        for tag, prs in self.pairs.items():
            ts = [a.elapsed_time(b) for a, b in prs]
            out[tag] = (len(ts), sum(ts) / len(ts))
        return out
