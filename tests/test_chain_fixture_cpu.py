"""The committed oracle-chain fixture (tests/golden/chain_oracle.json.gz) is what the oracle chain computes: the
'sparse' sets are recomputed here (cheap: ~0.4 s per frame) and compared -- detections within 1e-4 (fp32 CPU
convolutions may differ by ulps between machines / thread counts), the same chosen instance, rect, cells, A*
paths and costs.  The 300-detection sets take ~10 s per frame in the pure-Python findContours and are checked on
their first frame only."""
import pytest
import torch

from tests.chain_util import compare, frame_batch, load_fixture, oracle_frame, oracle_sequence, weights


def _same(got, want):
    c = compare(got, want, f32=True)
    assert c["det_same"], c
    assert c["chosen"] and c["cells"] and c["rect"] and c["paths"], c


def test_sparse_chain_fixture_recomputes():
    torch.set_num_threads(4)
    arch, fw = weights("sparse")
    want = load_fixture("chain/sparse")
    got = oracle_sequence(arch, fw, frame_batch(21, len(want)))
    for g, w in zip(got, want):
        _same(g, w)
    assert sum(w["chosen"] >= 0 for w in want) >= len(want) // 2
    nd = sorted(w["det"].shape[0] for w in want)  # the regime: a few detections per frame (32 frames: median 2,
    assert nd[len(nd) // 2] <= 5 and nd[-1] <= 16      # one frame with 12)


def test_c4_sparse_fixture_is_the_per_shard_replay():
    from oracle import nav as onav
    from vision_assist_amd.shard import shard_indices
    torch.set_num_threads(4)
    arch, fw = weights("sparse")
    want = load_fixture("c4/sparse")
    for r in range(2):
        pf = onav.PathFinderOracle()
        for i in shard_indices(len(want), 2, r):
            _same(oracle_frame(arch, fw, frame_batch(7000 + i, 1), pf), want[i])


@pytest.mark.slow
@pytest.mark.parametrize("regime", ["dense", "dense_box"])
def test_dense_chain_fixture_first_frame(regime):
    from oracle import nav as onav
    torch.set_num_threads(4)
    arch, fw = weights(regime)
    want = load_fixture(f"chain/{regime}")[0]
    _same(oracle_frame(arch, fw, frame_batch(21, 1), onav.PathFinderOracle()), want)
