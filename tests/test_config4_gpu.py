"""BASELINE configs[4] as a sharded fit at its own size, on one MI355X: SVD nFactors=256 on
the synthetic 10M users x 1M items x ~1e9 ratings set (rs_synth, seed 20250826), library defaults, 8 shards
through the in-process group with the exchange bench.py's strong_scaling and rs_svd_fit_multi run there
(RS_EXCHANGE_QDELTA: user ranges, 16 merges per epoch of the ranks' weighted item moves, fp16 wire), beside
the whole set fitted by one plan from the same factors.  Reference loop: core/svd.go:92-130.

About three and a half minutes on the box (generation ~35 s, the two plans ~55 s, 2 x 20 epochs); progress lines
go to the terminal so the run never looks silent.  Bound: within 0.005 of the whole-set fit after
10 epochs and after 20 (a default Fit, svd.go:66); round 6 measured 0.6127 / 0.5910 against 0.6081 / 0.5901.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu



@pytest.mark.timeout(900)
def test_config4_sharded_full_size(request):
    import config4_fit as C
    tr = request.config.pluginmanager.get_plugin("terminalreporter")
    say = (lambda *a: tr.write_line("  [configs[4]] " + " ".join(str(x) for x in a))) if tr else (lambda *a: None)
    out = C.run(C.parse(["--epochs", "20", "--exchange", "qdelta"]), say=say)
    whole, sh = out["whole"], out["sharded"]
    assert out["nnz_train"] > 9.9e8 and out["n_users"] == 10_000_000 and out["n_items"] == 1_000_000
    assert sh["finite"] and all(np.isfinite(x) for x in sh["rmse_per_epoch"])
    for ep in (10, 20):
        e_sh, e_whole = sh["rmse_per_epoch"][ep - 1], whole["rmse_per_epoch"][ep - 1]
        say(f"held-out RMSE after {ep} epochs: sharded {e_sh:.4f}, whole set {e_whole:.4f}")
        assert e_sh < 0.95
        assert abs(e_sh - e_whole) <= 0.005, (ep, e_sh, e_whole)
    assert all(b < a for a, b in zip(sh["rmse_per_epoch"], sh["rmse_per_epoch"][1:]))  # falls every epoch
