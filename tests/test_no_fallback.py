"""The product path is the HIP engine only: no CPU fallback, no oracle import."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "time-warp_amd")


def test_product_never_imports_oracle():
    for dirpath, _, files in os.walk(PKG):
        for f in files:
            if f.endswith((".py", ".hip", ".cpp", ".h")):
                src = open(os.path.join(dirpath, f)).read()
                assert not re.search(r"^\s*(import|from)\s+oracle\b", src, re.M), f
                assert "libtw_oracle" not in src and "timedt_oracle" not in src, f


def test_engine_fails_loudly_without_device():
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from timewarp.engine import Engine, EngineError

    with pytest.raises(EngineError, match="no HIP device"):
        Engine(0)
