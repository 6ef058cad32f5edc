"""GPU parity of the full FeatureExtractor map (a3) and the Flink rule scores ((f) rank 2) —
fd_features_full_device vs oracle/fmap_ref.py on the oracle feature state's raw features, same seeded
stream, extended profiles with nulls, unknown users / merchants, context with NaNs.
Bars: every column bit-exact except amount_log (device log, <= 1 ulp) and distance_to_merchant_km
(device sin/cos/atan2, 1e-9 relative); rule scores and codes bit-exact. Parity vs Java unpinned."""
import numpy as np
import pytest

from fdengine import FraudEngine, synth
from fdengine._native import CTX_FIELDS, RULE_DTYPE, TXN_FIELDS
from oracle import fmap_ref as R
from oracle.features_c import OracleFeatureState

pytestmark = pytest.mark.gpu


def _setup(engine, n_users, mode):
    pop = synth.population(n_users, 150, seed=n_users + 3)
    U, M = pop["users"], pop["merchants"]
    cap = 4 * n_users + 4096
    engine.state_init(cap, mode, 8)
    engine.load_users(U["key"], U["avg_amount"], U["account_age_days"], U["device_fp"])
    engine.load_merchants(M["fraud_rate"], M["risk_multiplier"])
    ue = synth.users_ext(pop)
    keep = np.random.default_rng(1).random(n_users) < 0.9  # some loaded users without extended fields
    engine.load_users_ext(ue["key"][keep], **{k: v[keep] for k, v in ue.items() if k != "key"})
    me = synth.merchants_ext(pop)
    n_me = 140  # merchants 140..149 have no extended profile
    engine.load_merchants_ext(n_me, **{k: v[:n_me] for k, v in me.items()})
    pay, ref = synth.vocab_flags()
    engine.load_vocab(pay, ref)
    orc = OracleFeatureState(cap, mode, 8)
    orc.load_users(U["key"], U["avg_amount"], U["account_age_days"], U["device_fp"])
    orc.load_merchants(M["fraud_rate"], M["risk_multiplier"])
    users_ext = {int(k): {f: ue[f][i] for f in ue if f != "key"} for i, k in enumerate(ue["key"]) if keep[i]}
    mext = {k: v[:n_me] for k, v in me.items()}
    return pop, orc, users_ext, mext, pay, ref


@pytest.mark.parametrize("mode", [0, 1])
def test_feature_map_and_rules_match_oracle(engine, mode):
    import torch
    pop, orc, users_ext, mext, pay, ref = _setup(engine, 1500, mode)
    tx = synth.txn_stream(pop, 12000, seed=21 + mode, rate_per_s=2.0, unknown_user_frac=0.05,
                          unknown_merchant_frac=0.05)
    rng = np.random.default_rng(4)
    tx["hour"] = tx["hour"].copy()
    has_h = rng.random(len(tx["hour"])) < 0.6  # Transaction.hourOfDay present on 60 %
    tx["hour"][has_h] = rng.integers(0, 24, int(has_h.sum()))
    tx["weekend"] = tx["weekend"].copy()
    tx["weekend"][rng.random(len(tx["weekend"])) < 0.3] = 1
    tx["amount_cents"] = tx["amount_cents"].copy()
    tx["amount_cents"][::17] = (tx["amount_cents"][::17] // 1000) * 1000  # round amounts
    ctx = synth.txn_context(tx)
    M = pop["merchants"]
    try:
        engine.set_stream(torch.cuda.current_stream().cuda_stream)
        for a, b in [(0, 3000), (3000, 12000)]:
            n = b - a
            part = {k: v[a:b] for k, v in tx.items()}
            cpart = {k: v[a:b] for k, v in ctx.items()}
            dev = {f: torch.from_numpy(np.ascontiguousarray(part[f])).cuda() for f in TXN_FIELDS}
            dctx = {f: torch.from_numpy(np.ascontiguousarray(cpart[f])).cuda() for f in CTX_FIELDS}
            vec = torch.empty((n, 64), dtype=torch.float32, device="cuda")
            fmap = torch.empty((n, 64), dtype=torch.float64, device="cuda")
            rules = torch.empty((n, 24), dtype=torch.uint8, device="cuda")
            engine.features_full_device({f: t.data_ptr() for f, t in dev.items()},
                                        {f: t.data_ptr() for f, t in dctx.items()}, n, vec.data_ptr(),
                                        fmap.data_ptr(), rules.data_ptr())
            torch.cuda.synchronize()
            raw, rvec, vel5 = orc.run_ex(part)
            efm, erules = R.feature_map(part, cpart, raw, vel5, users_ext,
                                        {"fraud_rate": M["fraud_rate"], "risk_multiplier": M["risk_multiplier"]},
                                        mext, pay, ref)
            got = fmap.cpu().numpy()
            exact = [c for c in range(64) if c not in (1, 25)]
            np.testing.assert_array_equal(got[:, exact], efm[:, exact])
            np.testing.assert_array_max_ulp(got[:, 1], efm[:, 1], maxulp=1)
            np.testing.assert_allclose(got[:, 25], efm[:, 25], rtol=1e-9, equal_nan=True)
            gr = rules.cpu().numpy().reshape(-1).view(np.dtype(RULE_DTYPE))
            for f in ("tp_score", "fe_score", "tp_decision", "tp_risk", "fe_decision", "fe_risk"):
                np.testing.assert_array_equal(gr[f], erules[f], err_msg=f)
            # coverage: the rules actually vary
            assert len(np.unique(gr["tp_decision"])) >= 2 and len(np.unique(gr["fe_risk"])) >= 3
            assert np.isnan(got[:, 19]).any() and (~np.isnan(got[:, 43])).any()
    finally:
        engine.set_stream(None)
