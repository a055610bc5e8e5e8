"""The driver's round-end smoke (__graft_entry__.smoke: one LM step on cuda:0 against the C oracle) as a -m gpu test,
so that a change of the product defaults cannot leave it comparing two different solvers unnoticed."""
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


@pytest.mark.gpu
def test_graft_smoke():
    import __graft_entry__
    __graft_entry__.smoke()
