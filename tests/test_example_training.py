"""The training example (reference SAGE layer flow on SpGEMMFunction) runs and
its loss falls (GPU)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "examples"))


@pytest.mark.gpu
def test_training_loss_falls():
    import train_maxk_sage
    losses = train_maxk_sage.main(["--graph", "flickr", "--nodes", "4000", "--steps", "40",
                                   "--hidden", "64", "--maxk", "16", "--layers", "2",
                                   "--feat", "50", "--classes", "7"])
    assert all(l == l for l in losses)                  # finite
    assert min(losses[-5:]) < 0.8 * losses[0], losses
