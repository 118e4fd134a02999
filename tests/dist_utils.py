"""Spawn a gloo process group of ``world`` CPU ranks for multi-process tests."""
import os
import socket
import traceback

import torch
import torch.multiprocessing as mp


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(rank, world, port, fn, out_dir, args):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), OMP_NUM_THREADS="2")
    torch.set_num_threads(2)
    try:
        res = fn(rank, world, *args)
        torch.save(res, os.path.join(out_dir, f"rank{rank}.pt"))
    except Exception:
        with open(os.path.join(out_dir, f"rank{rank}.err"), "w") as fh:
            fh.write(traceback.format_exc())
        raise
    finally:
        from bcfl.parallel import dist as D
        D.shutdown()


def run_world(fn, world, out_dir, *args):
    os.makedirs(out_dir, exist_ok=True)
    port = free_port()
    mp.start_processes(_entry, args=(world, port, fn, out_dir, args), nprocs=world, join=True,
                       start_method="spawn")
    return [torch.load(os.path.join(out_dir, f"rank{r}.pt"), weights_only=True) for r in range(world)]
