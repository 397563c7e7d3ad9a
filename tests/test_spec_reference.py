"""Oracle PCM vs an independent float64 ISO 11172-3 synthesis (tests/spec_dsp.py).

The reference's conformance test compares against mpg123 with the ISO/IEC
11172-4 bars (compliance_test.go:28-45): limited = RMS < 4.62 LSB and
max <= 32; full = RMS < 0.289 and max <= 2.  mpg123 is absent here, so the
independent float64 synthesis stands in for it; the oracle must meet the
FULL bar on the reference's sample streams and on synthetic streams that
exercise mixed blocks and intensity stereo.
"""
import numpy as np
import pytest

import oracle
import spec_dsp
from mp3g import synth

FULL_RMS, FULL_MAX = 0.289, 2


def _check(got, want):
    d = (got.astype(np.int64) - want.astype(np.int64)).astype(np.float64)
    rms, mx = float(np.sqrt((d ** 2).mean())), float(np.abs(d).max())
    assert rms < FULL_RMS and mx <= FULL_MAX, (rms, mx)


@pytest.mark.parametrize("name", ["classic_lame.mp3", "mpeg2.mp3"])
def test_oracle_full_compliance_vs_float64(captured, name):
    g, c, want = captured[name]
    got = spec_dsp.spec_decode(g, c, oracle.tables()["synth_d"].astype(np.float64))
    _check(got, want)


@pytest.mark.parametrize("kw", [dict(p_mixed=0.5, p_is=0.6, p_event=0.1),
                                dict(lsf=True, p_is=0.5, p_event=0.1),
                                dict(mode=synth.MODE_MONO, p_mixed=0.5, p_event=0.1)])
def test_oracle_full_compliance_synthetic(kw):
    g, c, s = synth.synth_batch(1, 50, seed=21, **kw)
    want, _ = oracle.dsp_streams(g, c, s)
    got = spec_dsp.spec_decode(g, c, oracle.tables()["synth_d"].astype(np.float64))
    _check(got, want)
