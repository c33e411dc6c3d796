"""The step's deferred read-back (vloss.PendingReadback / LazySave, CPU): a save dict resolves on its
first read through every access path the reference's code uses -- ``save["pred"]``,
``Video(**save)`` keyword unpacking (train_tools.save_results), ``dict(save)``, iteration, ``in`` --
and the resolve runs once (the failure it carries raises once).  (json's C encoder reads a dict
subclass's storage directly; the saves hold numpy arrays, which json cannot encode anyway.)"""
import pytest

from factmx.models import vloss


class _Ready:
    def synchronize(self):
        pass


def _pending(nvid=2, fail=False):
    calls = {"fill": 0}

    def check():
        if fail:
            raise RuntimeError("GRU timeout")

    def fill(saves):
        calls["fill"] += 1
        for v, s in enumerate(saves):
            s["pred"] = [v, v]
            s["loss"] = {"loss": 1.5 + v}
    return vloss.PendingReadback(_Ready(), check, fill, nvid), calls


def test_lazy_save_access_paths():
    for access in (lambda s: s["pred"], lambda s: (lambda **kw: kw)(**s)["loss"], lambda s: dict(s)["pred"],
                   lambda s: list(s), lambda s: "pred" in s, lambda s: s.get("loss"),
                   lambda s: len(s), lambda s: sorted(s.items()), lambda s: {**s}["pred"]):
        p, calls = _pending()
        out = access(p.saves[1])
        assert out not in (None, 0, [], {}), out
        assert calls["fill"] == 1 and p.done
        assert p.saves[0]["pred"] == [0, 0] and p.saves[1]["loss"] == {"loss": 2.5}
        access(p.saves[0])
        assert calls["fill"] == 1
    vloss.resolve_pending()


def test_pending_resolved_by_next_forward_and_failure_raises_once():
    p, calls = _pending(fail=True)
    with pytest.raises(RuntimeError, match="GRU"):
        vloss.resolve_pending()
    assert p.done and not vloss._PENDING
    vloss.resolve_pending()          # nothing left: no second raise


def test_failed_readback_error_persists_on_every_read():
    p, _ = _pending(fail=True)
    with pytest.raises(RuntimeError, match="GRU"):
        p.saves[0]["pred"]
    for s in p.saves:                 # later reads name the real failure, not KeyError('pred')
        with pytest.raises(RuntimeError, match="GRU"):
            s["pred"]
        with pytest.raises(RuntimeError, match="GRU"):
            s.get("loss")
    vloss.resolve_pending()


def test_lazy_save_pickles_and_copies_as_plain_dicts():
    import copy
    import pickle
    p, calls = _pending()
    s = p.saves[1]
    out = pickle.loads(pickle.dumps(s))
    assert type(out) is dict and out == {"pred": [1, 1], "loss": {"loss": 2.5}} and calls["fill"] == 1
    p2, _ = _pending()
    d = copy.deepcopy(p2.saves[0])
    assert type(d) is dict and d["pred"] == [0, 0]
    assert type(copy.copy(p2.saves[1])) is dict
    vloss.resolve_pending()
