"""fsdkr_collect_first_error_multi (collect_many's per-session outcomes in one
call) equals fsdkr_collect_first_error session by session, on CPU: a
multi-session SessionSet of shape-correct sessions (random field values, no GPU)
with random verdict bytes, mostly valid, some sessions failing each check."""
import os
import random
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))


def test_multi_equals_per_session():
    import pack_many_cpu
    from fsdkr.batch import SessionSet
    sess = pack_many_cpu.fake_sessions(48, bits=2048)
    ss = SessionSet(sess, 256, 2048, staged=False)
    v = ss.verdicts()
    rnd = random.Random(5)
    ok = {"feldman": 1, "pdl": 7, "range": 1, "ped": 1, "ck": 1, "dlog": 3}
    for name, good in ok.items():
        arr = getattr(v, name)
        arr[:] = good
        for _ in range(max(1, len(arr) // 40)):   # a few failing or panicking instances
            arr[rnd.randrange(len(arr))] = rnd.choice([0, good & ~1, good | (2 if name in ("range", "ped", "ck") else 8)])
    multi = ss.first_errors(v)
    assert sorted(multi) == sorted(ss.row)
    variants = set()
    for s in ss.row:
        one = ss.first_error(s, v)
        m = multi[s]
        assert (m.variant, m.panic, list(m.f), m.keys_applied) == (one.variant, one.panic, list(one.f), one.keys_applied)
        variants.add(one.variant)
    assert len(variants) > 1   # the draw exercised more than the all-valid outcome
    assert np.all(v.feldman >= 0)
