"""The N>1 path on CPU: world_size-2 gloo processes, each owning half of an 8-shard index.

Each rank computes its shards' per-shard top-k (here with the oracle, since there is no GPU — the
device path is covered by the -m gpu tests), encodes them as libosknn hit keys, and runs the same
gather + coordinator-reduce code bench.py runs on the MI355X node (distributed.ShardExchange: one
all-gather of the keys, host reduce for host tensors).  Every rank must end with the oracle's global
TopDocs.merge(from, size) with shardIndex = global shard number."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

N_SHARDS, ROWS, DIM, K, NQ = 8, 300, 32, 10, 3


def _key(score, doc):
    u = np.float32(score).view(np.uint32).item()
    s = (~u & 0xFFFFFFFF) if u & 0x80000000 else (u | 0x80000000)
    return np.uint64((s << 32) | (0xFFFFFFFF - int(doc)))


def _expected(from_, size):
    from oracle import oracle as O
    qs = O.synth(0, NQ, DIM, 43, 3)
    out = []
    for q in qs:
        shard_hits = []
        for s in range(N_SHARDS):
            rows = O.synth(s * ROWS, ROWS, DIM, 42, 3)
            sc, dc, _ = O.exact_search(rows, q, K, 2)
            shard_hits.append((sc, dc))
        out.append(O.topdocs_merge(shard_hits, from_, size, list(range(N_SHARDS))))
    return qs, out


def _worker(rank, world, port, from_, size, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from opensearch_amd import distributed as D
        from oracle import oracle as O
        own = D.owned_shards(rank, N_SHARDS, world)
        s_pad = D.max_shards_per_rank(N_SHARDS, world)
        qs = O.synth(0, NQ, DIM, 43, 3)
        keys = torch.zeros((NQ, s_pad, K), dtype=torch.int64)
        counts = torch.zeros((NQ, s_pad), dtype=torch.int32)
        for j, s in enumerate(own):
            rows = O.synth(s * ROWS, ROWS, DIM, 42, 3)
            for qi in range(NQ):
                sc, dc, _ = O.exact_search(rows, qs[qi], K, 2)
                kk = np.array([_key(a, b) for a, b in zip(sc, dc)], np.uint64)
                keys[qi, j, : len(kk)] = torch.from_numpy(kk.view(np.int64))
                counts[qi, j] = len(kk)
        gi = []
        for r in range(world):
            o = D.owned_shards(r, N_SHARDS, world)
            gi += o + [2**31 - 1] * (s_pad - len(o))
        xchg = D.ShardExchange(world, s_pad, NQ, K, from_, size, torch.tensor(gi, dtype=torch.int32))
        res = xchg(keys)
        q.put((rank, [t.numpy().tolist() for t in res]))
    except Exception as e:   # surface the failure instead of letting the parent wait
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,from_,size", [(2, 0, 10), (2, 5, 8), (3, 0, 12)])
def test_gloo_gather_and_merge(world, from_, size):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, from_, size, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    _, expected = _expected(from_, size)
    for rank in range(world):
        assert not isinstance(results[rank], str), results[rank]
        scores, docs, shard, count, total, mx = results[rank]
        for qi, (es, ed, esh, etot, emx) in enumerate(expected):
            n = len(ed)
            assert count[qi] == n
            assert docs[qi][:n] == list(ed) and shard[qi][:n] == list(esh)
            assert np.array_equal(np.float32(scores[qi][:n]), es)
            assert total[qi] == etot and np.float32(mx[qi]) == np.float32(emx)


def test_shard_ownership_is_contiguous_and_complete():
    from opensearch_amd import distributed as D
    for world in [1, 2, 3, 4, 8]:
        owned = [D.owned_shards(r, 8, world) for r in range(world)]
        assert sorted(s for o in owned for s in o) == list(range(8))
        assert all(o == list(range(o[0], o[0] + len(o))) for o in owned if o)


def test_shard_search_merge_checks_the_device_limits_before_any_collective():
    """The Python step refuses a shape beyond the communicator's device limits at construction (world > 1),
    with the call to make, instead of a refused, poisoning collective later."""
    from opensearch_amd import distributed as D

    class _Comm:
        world, device_limits = 2, D.DEFAULT_DEVICE_LIMITS

        def fits_device_limits(self, nq, k, spr):
            return D.DeviceComm.fits_device_limits(self, nq, k, spr)

    with pytest.raises(ValueError, match="set_device_limits"):
        D.ShardSearchMerge(_Comm(), None, 1, 2, 10, 0, 10, device=0)
