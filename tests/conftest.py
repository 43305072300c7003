import os
import sys

import pytest

# ct-add's host-side exponent bounds are verified against the device exponents in every test
# (fate_amd.paillier.CHECK_EBOUND); set before fate_amd is imported
os.environ.setdefault("FPHE_CHECK_EBOUND", "1")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP (MI355X) device")


def pytest_collection_modifyitems(config, items):
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no HIP device")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


# every latency kernel on (for any test-sized call) or every one off: parity tests that take
# `kernel_path` meet the oracle through both kernels of each op (fphe_ctx_set_option)
KERNEL_PATHS = {
    "latency": dict(wide_decrypt_max=1 << 20, wide_encrypt_max=1 << 20, wide_kh_encrypt_max=1 << 20,
                    wide_squeeze_max=1 << 20),
    "throughput": dict(wide_decrypt_max=0, wide_encrypt_max=0, wide_kh_encrypt_max=0, wide_squeeze_max=0),
}


@pytest.fixture(params=sorted(KERNEL_PATHS))
def kernel_path(request):
    """Runs the test with the latency kernels (wide_dev.h) or the throughput kernels the bench
    times (k_encrypt27, k_pow_half27, k_pow_half27<., ., true, true>, fphe_sqmul)."""
    from fate_amd import paillier as P
    with P.path_options(**KERNEL_PATHS[request.param]):
        yield request.param
