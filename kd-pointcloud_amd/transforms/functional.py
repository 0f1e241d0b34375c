"""Reference: transforms/functional.py:16-32."""
import torch


def to_tensor(array):
    """(N, C) numpy array -> (C, N) tensor sharing its memory (transpose first)."""
    assert len(array.shape) == 2
    return torch.from_numpy(array.transpose((1, 0)))
