#!/usr/bin/env python
"""Which Python call sites issue tensor copies (the runtime's __amd_rocclr_copyBuffer kernels) in
a bench round: Tensor.copy_ / clone / contiguous (when it copies) / to / torch.cat are wrapped and
tallied by issuing bcfl frame, call count and bytes moved, over the timed rounds of a one-client
(--clients 1) or multi-client federation.

    python scripts/copy_census.py [--clients 1] [--rounds 2]
"""
import argparse
import collections
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

TALLY = collections.Counter()
BYTES = collections.Counter()
ON = [False]


def _where():
    for fr in reversed(traceback.extract_stack()[:-2]):
        if "/bcfl/" in fr.filename and "copy_census" not in fr.filename:
            return f"{os.path.relpath(fr.filename)}:{fr.lineno} {fr.name}"
    return "?"


def _wrap(owner, name, nbytes_of):
    orig = getattr(owner, name)

    def w(*a, **k):
        out = orig(*a, **k)
        if ON[0]:
            nb = nbytes_of(a, out)
            if nb:
                key = (name, _where())
                TALLY[key] += 1
                BYTES[key] += nb
        return out
    setattr(owner, name, w)


def _op_census(fed, rounds):
    """Device-side census: every op whose GPU work includes a runtime copy kernel / memcpy,
    with the chain of enclosing ops (torch.profiler cpu_parent links; Python stacks are not
    recorded by this build), counted per round."""
    import torch
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        for r in range(1, rounds + 1):
            fed.run_round(r)
        torch.cuda.synchronize()
    chains = collections.Counter()
    us = collections.Counter()
    names = collections.Counter()
    for ev in prof.events():
        ks = [k for k in getattr(ev, "kernels", []) or []]
        hit = [k for k in ks if "copyBuffer" in k.name or "Memcpy" in k.name or "memcpy" in k.name]
        if not hit:
            continue
        chain, p = [], ev
        while p is not None and len(chain) < 6:
            chain.append(p.name + (str(p.input_shapes[:2]) if p is ev and p.input_shapes else ""))
            p = p.cpu_parent
        key = " <- ".join(chain)
        chains[key] += len(hit)
        us[key] += sum(k.duration for k in hit)
        for k in hit:
            names[k.name] += 1
    print("copy kernels by name:", dict(names))
    print(f"{'per round':>9} {'us/round':>9}  op chain")
    for key, n in sorted(chains.items(), key=lambda kv: -us[kv[0]])[:40]:
        print(f"{n / rounds:9.1f} {us[key] / rounds:9.1f}  {key}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=1)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--model", default="bert-base")
    ap.add_argument("--device", default="auto")
    ap.add_argument("--transport", default="auto", help="gossip transport (loopback = the N=1 bench's)")
    ap.add_argument("--lanes", type=int, default=0)
    ap.add_argument("--torch-prof", action="store_true",
                    help="GPU: attribute runtime copy kernels to the ops that issued them")
    a = ap.parse_args()
    import bcfl  # noqa: F401
    import torch
    from bcfl.config import get_preset
    from bcfl.fl import Federation

    def nb_out(args, out):
        return out.numel() * out.element_size() if torch.is_tensor(out) else 0

    def nb_copy(args, out):
        return args[0].numel() * args[0].element_size() if torch.is_tensor(args[0]) else 0

    def nb_contig(args, out):
        return (out.numel() * out.element_size()) if torch.is_tensor(out) and out.data_ptr() != args[0].data_ptr() else 0

    _wrap(torch.Tensor, "copy_", nb_copy)
    _wrap(torch.Tensor, "clone", nb_out)
    _wrap(torch.Tensor, "contiguous", nb_contig)
    _wrap(torch, "cat", nb_out)
    _wrap(torch.Tensor, "to", lambda a, o: (o.numel() * o.element_size())
          if torch.is_tensor(o) and o is not a[0] else 0)
    cfg = get_preset("baseline3_learnable", num_clients=a.clients, num_rounds=a.rounds + 1,
                     global_test_samples=125 * a.clients, out_dir="runs/census",
                     reference_prints=False, model=a.model, device=a.device,
                     gossip_transport=a.transport,
                     client_lanes=a.lanes or (a.clients if a.transport == "loopback" else 0))
    fed = Federation(cfg, verbose=False)
    fed.run_round(0)
    fed.drain()
    ON[0] = True
    if a.torch_prof and torch.cuda.is_available():
        _op_census(fed, a.rounds)
    else:
        for r in range(1, a.rounds + 1):
            fed.run_round(r)
    fed.drain()
    ON[0] = False
    print(f"{'calls/round':>11} {'MB/round':>9}  op  issuing frame")
    for key, n in sorted(TALLY.items(), key=lambda kv: -BYTES[kv[0]])[:40]:
        print(f"{n / a.rounds:11.1f} {BYTES[key] / a.rounds / 1e6:9.1f}  {key[0]:10s} {key[1]}")


if __name__ == "__main__":
    main()
