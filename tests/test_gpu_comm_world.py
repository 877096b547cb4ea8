"""The multi-rank exchange of osk_comm.hip at world 2, 3 and 8, on ONE GPU.

RCCL refuses two ranks on one device, so the testing build's loopback transport
(`osk_comm_init_loopback`, libosknn_testing.so) stands in for ncclAllGather: every rank is its own
process, stages its shards on the box's one GPU and runs exactly the world > 1 code of
`osk_shards_search_merge_device` / `osk_shards_search_merge` — per-call exchange blocks (lists padded
to shards-per-rank, header, shard indices), the gather on the communicator's exchange stream, and the
device coordinator reduce with the cross-rank header check.  Only the byte transport differs from the
8-GPU node.

* parity: the merged hits of every rank equal the N = 1 oracle merge (per-shard exactSearch +
  TopDocs.merge with shardIndex = global shard number) bit for bit, for both entries, from/size cuts
  and a k = 100 call that takes the merge_rank reduce;
* a rank that recreates its view between calls (a refresh on one node only) still merges correctly —
  the shard indices travel with every call, nothing is cached per (communicator, view);
* ranks that issue different calls (queries in another order, another from, another batch size on the
  host entry, batches that differ only in their last query) get count −1 and a poisoned communicator
  (OSK_ERR_INVALID), not a merge of unrelated lists; a poisoned communicator's later device calls still
  issue their collective (no rank may refuse on a flag the previous reduce writes asynchronously) and
  report count −1;
* one process driving several local devices (osk_comm_init_all; the testing build's
  osk_comm_init_all_loopback maps its n "devices" to the one GPU and replaces the grouped all-gather by
  device copies): the multi-device code of the host entry at n = 2 and 4 equals the oracle merge.

Reference semantics: S/action/search/SearchPhaseController.java:224-253 (mergeTopDocs, setShardIndex),
S/action/search/AbstractSearchAsyncAction.java:262-268 (one request per shard copy, loop index =
shardIndex).
"""
import multiprocessing as mp
import os
import traceback
import uuid

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

N_SHARDS = 8
DIM, SIM, SEED, DIST = 100, 2, 77, 3   # COSINE over L2-normalised Irwin–Hall rows
SIZES = [2500 + 611 * s for s in range(N_SHARDS)]
ROW0 = np.concatenate([[0], np.cumsum(SIZES)]).astype(np.int64)
# (n_queries, k, from, size, entry, query seed)
CALLS = [(1, 10, 0, 10, "device", 5), (3, 10, 2, 8, "device", 6), (2, 30, 5, 20, "device", 7),
         (4, 10, 0, 10, "host", 8), (1, 100, 0, 100, "device", 9), (2, 12, 0, 12, "host", 10)]


def _queries(nq, qseed):
    return O.synth(0, nq, DIM, 1000 + qseed, DIST)


def _worker(rank, world, name, mode, out_q):
    try:
        import ctypes as C

        import torch

        from opensearch_amd import _lib, distributed as D
        from opensearch_amd._lib import check, ptr
        with _lib.testing():
            L = _lib.lib()
            shards = D.owned_shards(rank, N_SHARDS, world)
            spr = D.max_shards_per_rank(N_SHARDS, world)
            segs = []
            for s in shards:
                h = C.c_void_p()
                check(L.osk_seg_synth(0, SIZES[s], DIM, _lib.FLOAT32, SIM, SEED, DIST, int(ROW0[s]), C.byref(h)))
                segs.append(h.value)

            def make_view():
                arr = (C.c_void_p * len(segs))(*segs)
                seg_shard = np.arange(len(segs), dtype=np.int32)
                base = np.zeros(len(segs), np.int32)
                sidx = np.asarray(shards, np.int32)
                v = C.c_void_p()
                check(L.osk_view_create(arr, len(segs), ptr(seg_shard), ptr(base), len(segs), ptr(sidx), C.byref(v)))
                return v

            view = make_view()
            comm = D.DeviceComm.init_loopback(0, rank, world, name)
            if mode == "over":
                comm.set_device_limits(1, 10, spr)
            else:   # (every rank alike: the device entry's fixed exchange block)
                comm.set_device_limits(165, 100, spr)
            stream = torch.cuda.Stream()

            def device_call(nq, k, from_, size, qs, spr=spr):
                dq = torch.from_numpy(_queries(nq, qs)).cuda()
                torch.cuda.synchronize()
                # (check_limits off: these calls test the library's own refusal, past the Python-side check)
                step = D.ShardSearchMerge(comm, view, spr, nq, k, from_, size, device=0, check_limits=False)
                res = step(dq.data_ptr(), stream.cuda_stream)
                stream.synchronize()
                return [t.cpu().numpy().copy() for t in res]

            results = []
            if mode in ("parity", "recreate"):
                for i, (nq, k, from_, size, entry, qs) in enumerate(CALLS):
                    if mode == "recreate" and rank == 1 and i % 2 == 1:   # this rank alone refreshes
                        check(L.osk_view_release(view))
                        view = make_view()
                    if entry == "device":
                        results.append(device_call(nq, k, from_, size, qs))
                    else:
                        results.append(list(D.shards_search_merge(comm, [view], _queries(nq, qs), k, from_, size)))
            elif mode == "misorder":
                # rank 0 issues query A then B, rank 1 B then A: the first call's blocks differ
                order = (5, 6) if rank == 0 else (6, 5)
                first = device_call(1, 10, 0, 10, order[0])
                rc, info = comm.status()
                # the next call still runs its collective on every rank (sticky flag → count −1)
                second = device_call(1, 10, 0, 10, order[1])
                results = [int(first[3][0]), int(first[4][0]), rc, info, int(second[3][0])]
            elif mode == "lastq":
                # 165 queries × 100 dims = 16,500 words: the batches differ in the last query only
                qs = _queries(165, 5)
                if rank == 1:
                    qs[-1] = qs[-1][::-1].copy()
                dq = torch.from_numpy(qs).cuda()
                torch.cuda.synchronize()
                step = D.ShardSearchMerge(comm, view, spr, 165, 10, 0, 10, device=0)
                res = step(dq.data_ptr(), stream.cuda_stream)
                stream.synchronize()
                rc, info = comm.status()
                results = [res[3].cpu().numpy().copy(), rc]
            elif mode == "devnq":
                # device entry, another batch size on rank 1: the block gather has the communicator's fixed
                # size on both ranks (no RCCL count mismatch), the header check reports count −1 on both
                nq = 1 if rank == 0 else 2
                first = device_call(nq, 10, 0, 10, 5)
                rc, info = comm.status()
                results = [first[3].tolist(), rc, info]
            elif mode == "devk":
                # device entry, another k on rank 1 (same batch): also only a header difference
                first = device_call(1, 10 if rank == 0 else 12, 0, 10, 5)
                rc, info = comm.status()
                results = [first[3].tolist(), rc, info]
            elif mode == "over":
                # rank 1 passes a batch beyond the limits (1 query): it still issues the collective (with a
                # refusal header) and returns OSK_ERR_INVALID; rank 0's call reports count −1
                nq = 1 if rank == 0 else 2
                try:
                    first = device_call(nq, 10, 0, 10, 5)
                    results = ["ok", first[3].tolist()]
                except _lib.OskError as e:
                    stream.synchronize()
                    results = [e.code, str(e)]
                rc, info = comm.status()
                results += [rc, info[0]]
            elif mode in ("badspr", "badfrom"):
                # rank 1's own arguments are wrong (its view holds more shards than the shards_per_rank it
                # passes / a negative from): it must still issue the all-gather (refusal header), so rank 0 is
                # not left waiting in it; rank 1 returns OSK_ERR_INVALID, rank 0 reports count −1
                bad = rank == 1
                try:
                    if mode == "badspr":
                        first = device_call(1, 10, 0, 10, 5, spr=len(shards) - 1 if bad else spr)
                    else:
                        first = device_call(1, 10, -1 if bad else 0, 10, 5)
                    results = ["ok", first[3].tolist()]
                except _lib.OskError as e:
                    stream.synchronize()
                    results = [e.code, str(e)]
                rc, info = comm.status()
                results += [rc, info[0]]
            elif mode == "misnq":
                # host entry, another batch size on rank 1: caught by the fixed-size call agreement before
                # the (differently sized) block gather
                nq = 2 if rank == 0 else 3
                try:
                    D.shards_search_merge(comm, [view], _queries(nq, 5), 10, 0, 10)
                    results = ["no error"]
                except _lib.OskError as e:
                    results = [e.code, str(e)]
            elif mode == "misfrom":
                # host entry, same block size, another `from` on rank 1
                from_ = 0 if rank == 0 else 2
                try:
                    D.shards_search_merge(comm, [view], _queries(2, 5), 10, from_, 8)
                    results = ["no error"]
                except _lib.OskError as e:
                    results = [e.code, str(e)]
            comm.close()
            check(L.osk_view_release(view))
            for h in segs:
                check(L.osk_seg_release(C.c_void_p(h)))
        out_q.put((rank, results))
    except BaseException:
        out_q.put((rank, "ERROR " + traceback.format_exc()))


def _run(world, mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    name = f"/osk_lb_{os.getpid()}_{uuid.uuid4().hex[:10]}"
    procs = [ctx.Process(target=_worker, args=(r, world, name, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            r, res = q.get(timeout=240)
            out[r] = res
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
        try:
            os.unlink("/dev/shm" + name)
        except OSError:
            pass
    for r in range(world):
        assert not (isinstance(out[r], str) and out[r].startswith("ERROR")), out[r]
    return out


def _oracle(nq, k, from_, size, qs):
    queries = _queries(nq, qs)
    want = []
    for i in range(nq):
        lists = []
        for s in range(N_SHARDS):
            rows = O.synth(int(ROW0[s]), SIZES[s], DIM, SEED, DIST)
            lists.append(O.exact_search(rows, queries[i], k, SIM)[:2])   # totalHits counts all k per shard
        want.append(O.topdocs_merge(lists, from_, size, list(range(N_SHARDS))))
    return want


@pytest.fixture(scope="module")
def expected():
    return [_oracle(nq, k, f, sz, qs) for (nq, k, f, sz, _, qs) in CALLS]


def _check(results, expected):
    for (nq, k, from_, size, entry, _), got, want in zip(CALLS, results, expected):
        sc, dc, sh, cnt, tot, mx = got
        for i in range(nq):
            es, ed, esh, et, em = want[i]
            n = int(cnt[i])
            assert n == len(ed), (entry, k, i)
            assert np.array_equal(dc[i, :n], ed) and np.array_equal(sh[i, :n], esh), (entry, k, i)
            assert np.array_equal(sc[i, :n].view(np.uint32), es.view(np.uint32)), (entry, k, i)
            assert int(tot[i]) == et and np.float32(mx[i]).view(np.uint32) == np.float32(em).view(np.uint32)


@pytest.mark.parametrize("world", [2, 3, 8])
def test_world_n_merge_equals_oracle(world, expected):
    out = _run(world, "parity")
    for r in range(world):
        _check(out[r], expected)


def test_one_rank_recreates_its_view_between_calls(expected):
    out = _run(2, "recreate")
    for r in range(2):
        _check(out[r], expected)


def test_misordered_calls_poison_the_communicator():
    out = _run(2, "misorder")
    for r in range(2):
        count, total, rc, info, second = out[r]
        assert count == -1 and total == -1
        assert rc == -1 and info[0] == 1 and info[1] == 1 and info[2] == 1 and info[3] == 1
        assert second == -1   # the next call ran its collective; its reduce reports the sticky poison


def test_mismatched_from_fails_the_host_entry():
    out = _run(2, "misfrom")
    for r in range(2):
        assert out[r][0] == -1 and "poisoned" in out[r][1], out[r]


def test_batches_differing_only_in_the_last_query_are_caught():
    out = _run(2, "lastq")
    for r in range(2):
        counts, rc = out[r]
        assert (counts == -1).all() and rc == -1, (r, counts[:4], rc)


@pytest.mark.parametrize("mode", ["devnq", "devk"])
def test_device_entry_mismatched_batch_or_k_gives_count_minus_one_no_hang(mode):
    """The device entry never waits on the host, so it cannot agree on the gather's size first: its block has
    the communicator's fixed size (osk_comm_set_device_limits) and a rank with another batch or k is a header
    difference — count −1 and a poisoned communicator on both ranks, not two all-gathers of different counts."""
    out = _run(2, mode)
    for r in range(2):
        counts, rc, info = out[r]
        assert all(c == -1 for c in counts), (r, counts)
        assert rc == -1 and info[0] == 1, (r, rc, info)


def test_device_entry_call_beyond_the_limits_is_refused_on_every_rank():
    out = _run(2, "over")
    assert out[0][0] == "ok" and out[0][1] == [-1], out[0]
    assert out[0][2] == -1 and out[0][3] == 1
    assert out[1][0] == -1 and "device limits" in out[1][1], out[1]
    assert out[1][2] == -1 and out[1][3] == 1


@pytest.mark.parametrize("mode", ["badspr", "badfrom"])
def test_device_entry_rank_local_argument_error_still_issues_the_gather(mode):
    """a rank whose own arguments fail (shards_per_rank below its view's shard count, a bad from)
    used to return before the all-gather and leave the other ranks inside it.  It now sends a refusal header:
    the other rank's reduce reports count −1 (no hang), the failing rank returns OSK_ERR_INVALID."""
    out = _run(2, mode)
    assert out[0][0] == "ok" and out[0][1] == [-1], out[0]
    assert out[0][2] == -1 and out[0][3] == 1
    assert out[1][0] == -1 and "refused on every rank" in out[1][1], out[1]


def test_mismatched_batch_size_fails_the_host_entry_before_the_gather():
    out = _run(2, "misnq")
    for r in range(2):
        assert out[r][0] == -1 and "poisoned" in out[r][1], out[r]


@pytest.mark.parametrize("n_local", [2, 4])
def test_init_all_multi_device_host_entry(n_local, expected):
    """One process, n local "devices" (all the one GPU): views[i] holds local device i's shards, the grouped
    exchange runs through the testing build's device-copy transport, the reduce on local device 0."""
    import ctypes as C

    from opensearch_amd import _lib, distributed as D
    from opensearch_amd._lib import check, ptr
    with _lib.testing():
        L = _lib.lib()
        segs, views = [], []
        for i in range(n_local):
            shards = D.owned_shards(i, N_SHARDS, n_local)
            mine = []
            for s in shards:
                h = C.c_void_p()
                check(L.osk_seg_synth(0, SIZES[s], DIM, _lib.FLOAT32, SIM, SEED, DIST, int(ROW0[s]), C.byref(h)))
                mine.append(h.value)
            arr = (C.c_void_p * len(mine))(*mine)
            seg_shard = np.arange(len(mine), dtype=np.int32)
            base = np.zeros(len(mine), np.int32)
            sidx = np.asarray(shards, np.int32)
            v = C.c_void_p()
            check(L.osk_view_create(arr, len(mine), ptr(seg_shard), ptr(base), len(mine), ptr(sidx), C.byref(v)))
            segs += mine
            views.append(v)
        comm = D.DeviceComm.init_all_loopback([0] * n_local)
        try:
            assert (comm.rank, comm.world, comm.n_local) == (0, n_local, n_local)
            results = [list(D.shards_search_merge(comm, views, _queries(nq, qs), k, f, sz))
                       for (nq, k, f, sz, _, qs) in CALLS]
            _check(results, expected)
            rc, info = comm.status()
            assert rc == 0 and info[0] == 0
        finally:
            comm.close()
            for v in views:
                check(L.osk_view_release(v))
            for h in segs:
                check(L.osk_seg_release(C.c_void_p(h)))
