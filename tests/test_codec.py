"""Kafka wire formats -- CPU tests of the host codecs in libcfk_als.so.

Expected bytes are built here independently with struct (big-endian, the layout java.io.DataOutputStream and
Kafka's IntegerSerializer / ShortSerializer produce), following FeatureMessageSerializer.java:27-37,
ListSerializer.java:72-84, FloatArraySerializer.java:15-24 and IdRatingPairMessageSerializer.java:24-33.
The out-block fan-out is pinned by the message counts SURVEY.md §2 measured on the reference's data/ at P=4
(tiny: 927 movie / 894 user messages per half; medium: 9,781 / 7,624).
"""
import struct

import numpy as np
import pytest


def _expected_feature_message(eid, deps, feats):
    b = struct.pack(">ii", eid, len(deps)) + struct.pack(f">{len(deps)}i", *deps)
    return b + struct.pack(">i", len(feats)) + struct.pack(f">{len(feats)}f", *feats)


def test_feature_message_bytes(cfk):
    feats = np.array([3.5, -0.25, 1e-30, 7.0], np.float32)
    for deps in ([], [7], [1, 5, 9, 2147483647], list(range(100))):
        got = cfk.encode_feature_message(42, deps, feats)
        assert got == _expected_feature_message(42, deps, feats.tolist())
        assert len(got) == 12 + 4 * len(deps) + 4 * len(feats)
        eid, d, f = cfk.decode_feature_message(got, len(feats))
        assert eid == 42 and d.tolist() == list(deps)
        assert f.view(np.uint32).tolist() == feats.view(np.uint32).tolist()


def test_feature_message_negative_id_and_special_floats(cfk):
    feats = np.array([np.inf, -np.inf, -0.0, np.float32(np.nan)], np.float32)
    got = cfk.encode_feature_message(-1, [-3], feats)
    # Float.floatToIntBits: every NaN is the canonical 0x7fc00000
    assert got[-4:] == bytes.fromhex("7fc00000")
    assert got[:12] == bytes.fromhex("ffffffff" "00000001" "fffffffd")
    assert got[16:28] == struct.pack(">fff", np.inf, -np.inf, -0.0)
    nan_payload = np.array([0x7f800001], np.uint32).view(np.float32)
    assert cfk.encode_feature_message(0, [], nan_payload)[-4:] == bytes.fromhex("7fc00000")


def test_feature_message_decode_rejects_inconsistent_lengths(cfk):
    msg = cfk.encode_feature_message(9, [1, 2, 3], np.ones(5, np.float32))
    with pytest.raises(cfk.ALSError, match="PARSE"):
        cfk.decode_feature_message(msg[:-1], 5)            # truncated
    with pytest.raises(cfk.ALSError, match="PARSE"):
        cfk.decode_feature_message(msg, 6)                 # NUM_FEATURES differs: deps length no longer fits
    with pytest.raises(cfk.ALSError, match="PARSE"):
        cfk.decode_feature_message(msg[:8], 5)             # shorter than id + list size + features
    bad = bytearray(msg)
    bad[4:8] = struct.pack(">i", 4)                        # list size disagrees with the inferred length
    with pytest.raises(cfk.ALSError, match="PARSE"):
        cfk.decode_feature_message(bytes(bad), 5)


def test_id_rating_pair_bytes(cfk):
    for eid, r in ((1, 5), (2649429, 3), (-1, 2), (0, -1), (2147483647, 32767)):
        got = cfk.encode_id_rating(eid, r)
        assert got == struct.pack(">ih", eid, r)
        assert cfk.decode_id_rating(got) == (eid, r)
    with pytest.raises(cfk.ALSError, match="PARSE"):
        cfk.decode_id_rating(b"\x00" * 5)


def _fanout_reference(ds, side, P):
    """Independent numpy restatement of the fan-out: per entity (ascending id), its partitions in
    first-appearance order over the arrival-order in-block, deps filtered by id % P."""
    blk = ds.shard_block(side, 1, 0)
    opp_ids = ds.ids(1 - side)
    msgs = []
    for r, eid in enumerate(blk["row_ids"]):
        ids = opp_ids[blk["col"][blk["row_ptr"][r]:blk["row_ptr"][r + 1]]]
        parts = []
        for i in ids:
            if i % P not in parts:
                parts.append(i % P)
        for p in parts:
            msgs.append((int(eid), int(p), [int(i) for i in ids if i % P == p]))
    return msgs


@pytest.mark.parametrize("which,P,counts", [("tiny", 4, (927, 894)), ("medium", 4, (9781, 7624)), ("tiny", 1, None),
                                            ("tiny", 7, None)])
def test_outblock_fanout(cfk, tiny_path, medium_path, which, P, counts):
    ds = cfk.Dataset.load_netflix(tiny_path if which == "tiny" else medium_path)
    k = 10
    for side in (0, 1):
        n = ds.counts()[side]
        F = np.random.default_rng(side).standard_normal((n, k)).astype(np.float32)
        buf, keys, offs = ds.feature_messages(side, P, F)
        if counts is not None:
            assert len(keys) == counts[side]
        ids = ds.ids(side)
        row_of = {int(i): r for r, i in enumerate(ids)}
        want = _fanout_reference(ds, side, P)
        assert len(want) == len(keys) and offs[-1] == len(buf)
        for m, (eid, p, deps) in enumerate(want):
            assert keys[m] == p
            msg = buf[offs[m]:offs[m + 1]]
            assert msg == _expected_feature_message(eid, deps, F[row_of[eid]].tolist())
    if which == "tiny" and P == 4:
        # about 64 KB of FeatureMessage payload per half at P=4, k=10
        assert 50_000 < len(buf) < 80_000
