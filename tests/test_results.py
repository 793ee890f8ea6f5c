"""CPU: stage checkpoints (SURVEY.md §5 checkpoint / resume) round-trip
bit-exactly through safetensors, with their metadata."""
import pytest
import torch

import tvr_amd


def test_results_round_trip(tmp_path):
    g = torch.Generator().manual_seed(0)
    mean = torch.randn(4, 3, 16, generator=g)
    cie = torch.randn(4, 3, generator=g).double()
    p = str(tmp_path / "stage.safetensors")
    tvr_amd.save_results(p, {"mean": mean, "cie": cie}, model="tiny", n_contexts=96, task="letter_to_caps")
    tensors, meta = tvr_amd.load_results(p)
    assert torch.equal(tensors["mean"], mean) and torch.equal(tensors["cie"], cie)
    assert tensors["cie"].dtype == torch.float64
    assert meta == {"model": "tiny", "n_contexts": 96, "task": "letter_to_caps"}


def test_results_refuse_empty(tmp_path):
    with pytest.raises(ValueError):
        tvr_amd.save_results(str(tmp_path / "x.safetensors"), {})
