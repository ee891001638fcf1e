"""seg.interleave_lanes: the laned op list's host enqueue order (the streams round-robin) keeps every dependency the
segment-by-segment list has -- each stream's own order, a lane op after the fork that opened its segment, a lane's
second fork after its first segment, joins after their lane's ops -- and puts the calling stream's next op ahead of
a lane's later ops."""
from types import SimpleNamespace as NS

from vision_assist_amd.seg import VA_OP_CONV, VA_OP_FORK, VA_OP_JOIN, interleave_lanes


def _op(name, lane=0, kind=VA_OP_CONV, n=0):
    return NS(kind=kind, lane=lane, a=NS(N=n), name=name)


def _laned():
    ops = [_op("A1"), _op("A2"), _op("fork1", kind=VA_OP_FORK, n=1)]
    ops += [_op(f"L1{c}", 1) for c in "abcd"]
    ops += [_op("B1"), _op("B2"), _op("fork2", kind=VA_OP_FORK, n=2)]
    ops += [_op(f"L2{c}", 2) for c in "ab"]
    ops += [_op("C1"), _op("C2"), _op("C3"), _op("fork2b", kind=VA_OP_FORK, n=2), _op("L2c", 2), _op("D1")]
    ops += [_op("join1", kind=VA_OP_JOIN, n=1), _op("join2", kind=VA_OP_JOIN, n=2)]
    return ops


def test_interleave_keeps_dependencies_and_feeds_the_calling_stream():
    ops = _laned()
    got, meta = interleave_lanes(ops, [o.name for o in ops])
    names = [o.name for o in got]
    assert meta == names and sorted(names) == sorted(o.name for o in ops)
    pos = {n: i for i, n in enumerate(names)}
    for s in (0, 1, 2):  # each stream's own order (forks / joins are the calling stream's)
        mine = [o.name for o in ops if (o.lane if o.kind == VA_OP_CONV else 0) == s]
        assert [n for n in names if n in mine] == mine
    for n in ("L1a", "L1b", "L1c", "L1d"):
        assert pos["fork1"] < pos[n] < pos["join1"]
    for n in ("L2a", "L2b"):
        assert pos["fork2"] < pos[n] < pos["fork2b"]
    assert pos["fork2b"] < pos["L2c"] < pos["join2"]
    # the calling stream is not held behind lane 1's whole segment
    assert pos["B1"] < pos["L1c"] and pos["B2"] < pos["L1d"]


def test_interleave_of_a_list_without_lanes_is_the_identity():
    ops = [_op(f"x{i}") for i in range(5)]
    got, _ = interleave_lanes(ops, [o.name for o in ops])
    assert [o.name for o in got] == [o.name for o in ops]
