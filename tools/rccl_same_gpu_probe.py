"""Development probe: can two processes form one RCCL communicator on the SAME GPU (the 1-GPU box)?
If RCCL accepts it, the engine's RCCL all-reduce path (sglm_set_comm_rccl, bench's rccl-engine) runs
at world 2 here; if it refuses (duplicate device), each rank reports the error.  Each rank fits a
small logit shard and prints its deviance.  usage: python tools/rccl_same_gpu_probe.py"""
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rank_main(rank: int, world: int, uid_path: str) -> int:
    sys.path.insert(0, ROOT)
    from sparkglm_amd import Engine
    if rank == 0:
        uid = Engine.rccl_unique_id()
        with open(uid_path + ".tmp", "wb") as f:
            f.write(uid)
        os.replace(uid_path + ".tmp", uid_path)
    else:
        t0 = time.time()
        while not os.path.exists(uid_path):
            if time.time() - t0 > 60:
                print(f"rank {rank}: no unique id", flush=True)
                return 2
            time.sleep(0.05)
        uid = open(uid_path, "rb").read()
    e = Engine(0)
    try:
        e.synth(0, rank * 200_000, 200_000, 64, 3)
        e.set_comm_rccl(world, rank, uid)
        f = e.fit_glm("binomial", "logit")
        st = e.stats()
        print(f"rank {rank}: iter {f.iter} deviance {f.deviance!r} comm {st['comm_path_name']}", flush=True)
    except Exception as exc:  # noqa: BLE001
        print(f"rank {rank}: {type(exc).__name__}: {exc}", flush=True)
        return 1
    finally:
        e.close()
    return 0


if __name__ == "__main__":
    if len(sys.argv) > 1:
        sys.exit(rank_main(int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]))
    world = 2
    d = tempfile.mkdtemp()
    uid = os.path.join(d, "uid")
    env = dict(os.environ, SGLM_COMM_TIMEOUT_S="60")
    ps = [subprocess.Popen([sys.executable, __file__, str(r), str(world), uid], env=env) for r in range(world)]
    rc = [p.wait(timeout=240) for p in ps]
    print("exit codes", rc)
    sys.exit(max(rc))
