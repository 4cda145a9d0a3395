"""The JPEG frame-decode oracle (oracle/jpeg_oracle.py, a restatement of libjpeg-turbo's islow IDCT,
fancy upsampling and YCbCr -> RGB) pinned against Pillow - the decoder the reference calls
(core/preprocessing/frame_loader.py:42-44) - and the library's host-side header parsing (no GPU)."""
import ctypes as C
import io

import numpy as np
import pytest
from PIL import Image

from helpers import jpeg_cases
from oracle import jpeg_oracle as J
from vcap import _native as N

CASES = jpeg_cases()


@pytest.mark.parametrize("name,data", CASES, ids=[c[0] for c in CASES])
def test_oracle_bit_exact_vs_pillow(name, data):
    ref = np.asarray(Image.open(io.BytesIO(data)).convert("RGB"))
    assert np.array_equal(J.decode(data), ref)


def test_probe_reports_size_and_refuses_progressive():
    lib = N.lib()
    w, h, c = C.c_int(), C.c_int(), C.c_int()
    name, data = CASES[0]
    assert lib.vcap_jpeg_probe(data, len(data), C.byref(w), C.byref(h), C.byref(c)) == 0
    assert (h.value, w.value, c.value) == (37, 53, 3)
    assert lib.vcap_jpeg_workspace_bytes(data, len(data), 4) > 0
    b = io.BytesIO()
    Image.open(io.BytesIO(data)).save(b, format="JPEG", progressive=True)
    p = b.getvalue()
    rc = lib.vcap_jpeg_probe(p, len(p), C.byref(w), C.byref(h), C.byref(c))
    assert rc < 0 and b"progressive" in lib.vcap_last_error()
    assert lib.vcap_jpeg_workspace_bytes(p, len(p), 1) == 0
    assert lib.vcap_jpeg_probe(b"not a jpeg", 10, C.byref(w), C.byref(h), C.byref(c)) < 0
