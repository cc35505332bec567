import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (HIP device); run with -m gpu')


@pytest.fixture(scope='session')
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no HIP device')
    return torch.device('cuda:0')


@pytest.fixture(autouse=True)
def _fresh_dropout_seed_source():
    """Each test starts without the process-wide dropout step counter
    (srf_set_seed_source): a training-step test attaches one, and the kernel tests
    that restate dropout masks (tests/torch_ref.py) assume the per-call seeds alone."""
    yield
    from srf_amd import ops, trainer_sr
    ops.check_faults()   # no grouped SDR recurrence of the test timed out (srf_set_fault_flag)
    if trainer_sr._SEED_COUNTERS:
        import torch
        from srf_amd import _lib
        torch.cuda.synchronize()
        _lib.check(_lib.lib().srf_set_seed_source(None), 'srf_set_seed_source')
        trainer_sr._SEED_COUNTERS.clear()
