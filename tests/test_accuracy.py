"""Ground-truth accuracy: the error classes of
reporter_amd.synth.classify_sequences, and a regression guard on the spec's
matching quality against the routes the synthetic vehicles drove (CPU
oracle; the GPU path is bit-identical to it)."""
from reporter_amd import synth


def test_classes_on_hand_sequences():
    twin = {2: {20}, 20: {2}, 3: {30}, 30: {3}}
    c = synth.classify_sequences([1, 2, 3, 4], [1, 2, 20, 2, 3, 4], twin)
    assert c["inserted_uturn"] == 2 and c["paired"] == 4
    c = synth.classify_sequences([1, 2, 3, 4], [1, 2, 7, 3, 4], twin)
    assert c["inserted_other"] == 1
    c = synth.classify_sequences([1, 2, 3, 4], [1, 2, 7, 3, 4], twin, at_outlier=lambda k0, k1: (k0, k1) == (1, 3))
    assert c["inserted_outlier"] == 1 and c["inserted_other"] == 0
    c = synth.classify_sequences([1, 2, 3, 4], [1, 3, 4], twin)
    assert c["dropped"] == 1
    c = synth.classify_sequences([1, 2, 3, 4], [1, 30, 4], twin)
    assert c["reverse"] == 1 and c["swap"] == 1
    c = synth.classify_sequences([1, 2, 3, 4], [9, 2, 3, 8, 7], twin)
    assert (c["start_missed"], c["start_extra"], c["end_missed"], c["end_extra"]) == (1, 1, 1, 2)
    c = synth.classify_sequences([1, 2], [5, 6], twin)
    assert c["no_overlap"] == 1 and c["paired"] == 0


def test_interior_accuracy_guard(small_graph, oracle):
    """City graph, config-2 noise: outside outlier columns the interior
    agreement stays above the north star's 99.9 % (round 3's forward-only
    same-edge rule gave ~95 %: U-turn excursions)."""
    b = synth.make_traces(small_graph, 150, 60, noise_sigma_m=15.0, accuracy=15.0, seed=21)
    orc = oracle.match_batch(oracle.Graph(small_graph), b, nthreads=4, keep_stages=True)
    poff, pedges = synth.true_paths(small_graph, 150, 60, noise_sigma_m=15.0, accuracy=15.0, seed=21)
    out = synth.outlier_points(small_graph, b["true_edge"], orc["ncand"], orc["cand_edge"], orc["cand_off"],
                               b["trace_off"], orc["gc"])
    agr = synth.segment_agreement(small_graph, poff, pedges, orc, trace_off=b["trace_off"], outlier=out)
    bd = agr["breakdown"]
    assert bd["driven_segments"] > 500
    assert bd["inserted_uturn"] <= 1
    assert bd["interior_agreement_outside_outliers"] >= 0.999, bd
    assert 0.9 < agr["segment_id_agreement"] <= 1.0
