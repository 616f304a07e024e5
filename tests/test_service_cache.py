"""The service's database cache (CPU, fake databases): reference counting
keeps a database open while any request holds a lease, a replaced file's
database closes when its last user leaves, threads share one entry."""
import os
import threading
import time

import pytest


class FakeDB:
    opened = []

    def __init__(self, path):
        self.path, self.closed = path, False
        FakeDB.opened.append(self)

    def close(self):
        assert not self.closed
        self.closed = True


@pytest.fixture()
def svc(monkeypatch):
    from patmatchdocker_amd import engine, service
    FakeDB.opened = []
    monkeypatch.setattr(engine.SequenceDatabase, "from_file", classmethod(lambda cls, p, device=0: FakeDB(p)))
    cache = service._DatabaseCache()
    yield service, cache
    cache.clear()


def test_lease_keeps_a_replaced_database_open(svc, tmp_path):
    _, cache = svc
    f = tmp_path / "a.seq"
    f.write_bytes(b">a\nACGT\n")
    with cache.lease(str(f)) as db1:
        os.utime(f, ns=(1, 1))
        f.write_bytes(b">a\nACGTT\n")
        with cache.lease(str(f)) as db2:
            assert db2 is not db1 and not db1.closed
        assert not db1.closed and not db2.closed
    assert db1.closed and not db2.closed
    cache.clear()
    assert db2.closed


def test_threads_share_one_entry(svc, tmp_path):
    _, cache = svc
    f = tmp_path / "b.seq"
    f.write_bytes(b">b\nACGT\n")
    seen = []

    def work():
        for _ in range(50):
            with cache.lease(str(f)) as db:
                assert not db.closed
                seen.append(db)
                time.sleep(0.0005)

    ts = [threading.Thread(target=work) for _ in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert len(FakeDB.opened) == 1 and len(set(map(id, seen))) == 1


def test_a_failed_open_is_retried_by_the_next_lease(svc, monkeypatch, tmp_path):
    """"reopen" retires the entry before it opens the file again; an open
    that raises leaves no entry behind, so the next lease opens again, and
    resident() never reports a retired entry (a closed entry
    stayed in the table and every later request got a database of None)."""
    from patmatchdocker_amd import engine
    _, cache = svc
    f = tmp_path / "c.seq"
    f.write_bytes(b">c\nACGT\n")
    with cache.lease(str(f)) as db1:
        pass
    assert cache.resident(str(f))
    calls = {"n": 0}

    def flaky(cls, p, device=0):
        calls["n"] += 1
        if calls["n"] == 1:
            raise RuntimeError("open failed")
        return FakeDB(p)

    monkeypatch.setattr(engine.SequenceDatabase, "from_file", classmethod(flaky))
    with pytest.raises(RuntimeError):
        with cache.lease(str(f), mode="reopen"):
            pass
    assert db1.closed and not cache.resident(str(f))
    with cache.lease(str(f), mode="cached") as db2:   # no entry: opens, whatever the mode
        assert db2 is not db1 and not db2.closed
    assert cache.resident(str(f)) and calls["n"] == 2
    with cache.lease(str(f)) as db3:
        assert db3 is db2
