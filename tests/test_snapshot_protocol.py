"""CPU: the sharded checkpoint / rescale protocol (fdengine.sharding.ShardedScorer.checkpoint / restore) at
world_size 2 over gloo, with a test backend whose "image" is the set of card keys it owns (the GPU image
format and its bit-exact resume are tested in tests/test_gpu_snapshot.py).

Bar: the manifest names every rank's image; restoring the world-2 checkpoint on 3 (and 1) shards gives every
card to exactly one new shard — its owner under shard_of — i.e. the key-group redistribution Flink does
on rescale (fl/FraudDetectionJob.java:112-136 externalized checkpoints)."""
import json
import os
import socket

import numpy as np
import pytest

from oracle import route_ref as R

WORLD = 2


class KeySetBackend:
    def __init__(self, keys):
        self.keys = np.asarray(keys, np.uint64)

    def snapshot(self, path, rank, world):
        with open(path, "w") as f:
            json.dump({"rank": rank, "world": world, "keys": [int(k) for k in self.keys]}, f)
        return os.path.getsize(path)

    def restore(self, path, rank, world):
        with open(path) as f:
            keys = np.array(json.load(f)["keys"], np.uint64)
        mine = keys[R.shard_of(keys, world) == rank]
        self.keys = np.union1d(self.keys, mine)
        return len(mine)


def _all_keys():
    rng = np.random.default_rng(3)
    return np.unique(rng.integers(1, 2**63, 5000, dtype=np.int64).astype(np.uint64))


def _worker(rank, port, outdir):
    import torch.distributed as dist
    from fdengine.sharding import ShardedScorer
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        keys = _all_keys()
        sc = ShardedScorer(KeySetBackend(keys[R.shard_of(keys, WORLD) == rank]), rank, WORLD)
        man = sc.checkpoint(outdir, step=7)
        # after the barrier inside checkpoint() the manifest exists on every rank
        assert os.path.exists(man)
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(120)
def test_world2_checkpoint_restores_on_any_world(tmp_path):
    import torch.multiprocessing as mp

    from fdengine.sharding import ShardedScorer, image_name, latest_checkpoint
    mp.spawn(_worker, args=(_free_port(), str(tmp_path)), nprocs=WORLD, join=True)
    man = latest_checkpoint(str(tmp_path))
    assert man is not None and man.endswith("checkpoint-00000007.json")
    doc = json.load(open(man))
    assert doc["world"] == 2 and doc["images"] == [image_name(7, r, 2) for r in range(2)]
    assert all(b > 0 for b in doc["bytes"])
    keys = _all_keys()
    for new_world in (3, 1):
        got = []
        for r in range(new_world):
            be = KeySetBackend([])
            n = ShardedScorer(be, r, new_world).restore(man)
            assert n == len(be.keys)
            assert (R.shard_of(be.keys, new_world) == r).all()
            got.append(be.keys)
        allk = np.concatenate(got)
        assert len(allk) == len(keys) and np.array_equal(np.sort(allk), keys)


def test_restore_rejects_foreign_manifest(tmp_path):
    from fdengine.sharding import ShardedScorer
    p = tmp_path / "checkpoint-00000001.json"
    p.write_text(json.dumps({"format": "other"}))
    with pytest.raises(ValueError, match="not an fdengine checkpoint"):
        ShardedScorer(KeySetBackend([]), 0, 1).restore(str(p))
