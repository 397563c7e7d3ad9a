"""The oracle's split of Frame.Decode at subbandSynthesis (CPU, no GPU).

orc_hybrid_streams (requantize .. frequencyInversion, frame.go:140-486)
followed by orc_synth_streams (subbandSynthesis, frame.go:630-688) must give
exactly the PCM and vVec state of the whole-frame oracle (orc_dsp_streams):
these two functions are the checker of the standalone polyphase entry point
mp3g_plan_synth_execute (tests/test_gpu_synth.py).
"""
import numpy as np
import pytest

import oracle
from mp3g import synth


@pytest.mark.parametrize("name", ["classic_lame.mp3", "mpeg2.mp3"])
def test_split_equals_whole_frame_files(captured, name):
    import mp3g
    g, c, want = captured[name]
    s = mp3g.streams_for([len(g)], mp3g.STATE_OUT)
    lines = oracle.hybrid_streams(g, c, s)
    pcm, so = oracle.synth_streams(g, lines, s)
    assert np.array_equal(pcm, want)
    _, so_ref = oracle.dsp_streams(g, c, s)
    assert np.array_equal(so["vvec"], so_ref["vvec"])


def test_split_equals_whole_frame_synthetic_with_state():
    import mp3g
    g, c, s = synth.synth_batch(3, 40, seed=5, p_mixed=0.2, p_is=0.3)
    # streams 0 and 2 start from a state: that of decoding their first 7 granules
    pre = mp3g.streams_for([7, 7, 7], mp3g.STATE_OUT)
    idx = np.concatenate([np.arange(int(x["first_granule"]), int(x["first_granule"]) + 7) for x in s])
    _, st = oracle.dsp_streams(g[idx], c[idx], pre)
    s = s.copy()
    s["flags"][[0, 2]] |= mp3g.STATE_IN
    s["flags"] |= mp3g.STATE_OUT
    want, so_ref = oracle.dsp_streams(g, c, s, state_in=st)
    lines = oracle.hybrid_streams(g, c, s, state_in=st)
    pcm, so = oracle.synth_streams(g, lines, s, state_in=st)
    assert np.array_equal(pcm, want)
    assert np.array_equal(so["vvec"], so_ref["vvec"])
    # the synthesis stage passes the IMDCT overlap through
    assert np.array_equal(so["store"][[0, 2]], st["store"][[0, 2]])
    assert not so["store"][1].any()
