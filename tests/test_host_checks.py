"""Host-side argument checks of the Python mirror that run before any native call (no GPU)."""
import numpy as np
import pytest

from spec_viterbi_amd.viterbi import DeviceBatch, DeviceModel, _result_arrays


def _model_stub(n=4):
    m = object.__new__(DeviceModel)  # no device model: the checks must raise before the C ABI
    m.n, m.S, m._h = n, 2, None
    return m


@pytest.mark.parametrize("offsets,symbols", [
    ([0, 3, 9], np.zeros(8, np.uint8)),            # offsets[-1] past the symbols
    ([0, 5, 3], np.zeros(8, np.uint8)),            # decreasing
    ([[0, 3]], np.zeros(8, np.uint8)),             # not 1-D
    ([], np.zeros(8, np.uint8)),                   # no entries
    ([0, 3], np.zeros((2, 4), np.uint8)),          # 2-D symbols
    ([0, 9], np.zeros(8, np.uint64)),              # uint64 path too
])
def test_viterbi_packed_rejects_bad_offsets(offsets, symbols):
    with pytest.raises(ValueError):
        _model_stub().viterbi_packed(np.asarray(offsets, np.uint64), symbols)


def test_result_arrays_checks_out():
    s, b = _result_arrays(None, 3, 4)
    assert s.shape == (3, 4) and s.dtype == np.float32 and b.shape == (3,) and b.dtype == np.int64
    good = (np.empty((3, 4), np.float32), np.empty(3, np.int64))
    assert _result_arrays(good, 3, 4)[0] is good[0]
    for bad in ((np.empty((3, 5), np.float32), good[1]), (good[0], np.empty(3, np.int32)),
                (np.empty((4, 3), np.float32).T, good[1])):
        with pytest.raises(ValueError):
            _result_arrays(bad, 3, 4)


def test_batch_read_checks_out():
    b = object.__new__(DeviceBatch)
    b.nseq, b.model, b._h = 2, _model_stub(4), None
    with pytest.raises(ValueError):
        b.read(out=(np.empty((2, 3), np.float32), np.empty(2, np.int64)))
