"""Checkpoints in the Hugging Face layout (``config.json`` + ``model.safetensors``), written async.

Reference behaviour: ``global_model.save_pretrained(dir)`` every round, overwriting,
fp32 (``src/Serverlesscase/serverless_NonIID_IMDB.py:305``: ``./my_albert_model2``), synchronously
inside the round; the server case never checkpoints; nothing is ever loaded back.

Here:
* ``<out>/global/`` (and ``<out>/client_<k>/`` with ``save_clients``) hold HF-named fp32 tensors,
  so ``transformers.AutoModelForSequenceClassification.from_pretrained(<out>/global)`` works;
  ``compat_save_path`` mirrors the reference's directory names.
* Saving is asynchronous: the fp32 master buffer is copied D2H on a side stream into a pinned
  buffer, and a background thread serialises it; if the writer is still busy the request is
  coalesced (the directory always holds the latest completed round, as the reference's
  overwrite semantics imply). A BERT-base round is ~0.1-0.3 s on MI355X, a synchronous 433 MB
  write would dominate it.
* ``state.json`` carries the round counter, dropout-RNG state and ledger tip for ``--resume``.
"""
from __future__ import annotations

import concurrent.futures as cf
import json
import os
import shutil
import struct
import threading
from typing import Any, Dict, List, Optional, Tuple

import numpy as np
import torch

_DT = {torch.float32: "F32", torch.bfloat16: "BF16", torch.float16: "F16", torch.int64: "I64",
       torch.int32: "I32"}


def hf_layout(model, flat) -> List[Tuple[str, int, Tuple[int, ...]]]:
    """(hf_name, element offset into the flat buffer, shape) for every trainable HF tensor."""
    base = flat.param.data_ptr()
    es = flat.param.element_size()
    out = []
    items = model.adapter_items() if getattr(model, "lora", False) else model.hf_items()
    for name, get, _ in items:
        t = get()
        off = (t.data_ptr() - base) // es
        if off < 0 or off + t.numel() > flat.numel:
            continue  # frozen tensor, not in the federated buffer
        out.append((name, int(off), tuple(t.shape)))
    return out


def write_safetensors(path: str, tensors: List[Tuple[str, np.ndarray]], metadata: Optional[Dict[str, str]] = None):
    header: Dict[str, Any] = {}
    off = 0
    for name, arr in tensors:
        n = arr.nbytes
        dt = {np.dtype("float32"): "F32", np.dtype("float16"): "F16", np.dtype("int64"): "I64",
              np.dtype("int32"): "I32", np.dtype("uint16"): "BF16"}[arr.dtype]
        header[name] = {"dtype": dt, "shape": list(arr.shape), "data_offsets": [off, off + n]}
        off += n
    if metadata:
        header["__metadata__"] = {k: str(v) for k, v in metadata.items()}
    hb = json.dumps(header, separators=(",", ":")).encode()
    hb += b" " * ((8 - len(hb) % 8) % 8)
    tmp = path + ".tmp"
    with open(tmp, "wb") as fh:
        fh.write(struct.pack("<Q", len(hb)))
        fh.write(hb)
        for _, arr in tensors:
            fh.write(memoryview(np.ascontiguousarray(arr)).cast("B"))
    os.replace(tmp, path)


def read_safetensors(path: str) -> Dict[str, torch.Tensor]:
    from safetensors.torch import load_file
    return load_file(path)


def save_dir(out_dir: str, model, flat_host: np.ndarray, layout, config: Dict[str, Any],
             metadata: Optional[Dict[str, str]] = None):
    os.makedirs(out_dir, exist_ok=True)
    tensors = [(n, flat_host[o:o + int(np.prod(s))].reshape(s)) for n, o, s in layout]
    write_safetensors(os.path.join(out_dir, "model.safetensors"), tensors,
                      {"format": "pt", **(metadata or {})})
    with open(os.path.join(out_dir, "config.json"), "w") as fh:
        json.dump(config, fh, indent=2, sort_keys=True)


def link_dir(src_dir: str, out_dir: str, config: Dict[str, Any]):
    """``out_dir`` gets the weights ``save_dir`` just wrote to ``src_dir`` (hard link, or a copy
    across filesystems). Writers replace files (tmp + rename), so a later save never changes a
    linked file in place."""
    os.makedirs(out_dir, exist_ok=True)
    src = os.path.join(src_dir, "model.safetensors")
    dst = os.path.join(out_dir, "model.safetensors")
    tmp = dst + ".tmp"
    if os.path.lexists(tmp):
        os.remove(tmp)
    try:
        os.link(src, tmp)
    except OSError:
        shutil.copyfile(src, tmp)
    os.replace(tmp, dst)
    with open(os.path.join(out_dir, "config.json"), "w") as fh:
        json.dump(config, fh, indent=2, sort_keys=True)


def dir_size_gb(path: str) -> float:
    """Reference ``get_dir_size`` (os.walk sum; E5's getsize-on-a-directory bug fixed)."""
    tot = 0
    for dp, _, fs in os.walk(path):
        for f in fs:
            fp = os.path.join(dp, f)
            if os.path.exists(fp):
                tot += os.path.getsize(fp)
    return tot / 1024 ** 3


class AsyncCheckpointer:
    """HF-layout checkpoints written off the critical path: each job's fp32 master is copied
    device->pinned host on a copy stream, then a writer thread serialises it. The compute stream
    waits (on the GPU, no host sync) for the copies before anything can overwrite a source buffer,
    so a checkpoint never mixes two rounds' weights. A save requested while the previous write is
    still running is skipped and counted (``skipped``)."""

    def __init__(self, model, flat, async_: bool = True):
        self.model, self.flat = model, flat
        self.layout = hf_layout(model, flat)
        self.config = model.hf_config()
        self.async_ = async_
        dev = flat.master.device
        self.cuda = dev.type == "cuda"
        self.pinned: List[torch.Tensor] = []
        self.snaps: List[torch.Tensor] = []   # device-side snapshots the D2H copies read
        self.stream = torch.cuda.Stream(device=dev) if self.cuda else None
        self.pool = cf.ThreadPoolExecutor(max_workers=1) if async_ else None
        self.future: Optional[cf.Future] = None
        self.skipped = 0
        self.saved = 0
        self.last_dir = None
        self._lock = threading.Lock()

    def busy(self) -> bool:
        return self.future is not None and not self.future.done()

    def _buf(self, i: int) -> torch.Tensor:
        while len(self.pinned) <= i:
            self.pinned.append(torch.empty(self.flat.numel, dtype=torch.float32,
                                           pin_memory=self.cuda))
        return self.pinned[i]

    def save(self, out_dirs: List[str], master: Optional[torch.Tensor] = None,
             metadata: Optional[Dict[str, str]] = None, state: Optional[Dict[str, Any]] = None,
             jobs: Optional[List[tuple]] = None, extra_files: Optional[Dict[str, Any]] = None) -> bool:
        """``jobs``: [(dirs, fp32 flat master)] (default: one job ``(out_dirs, master)``);
        ``state`` is written as ``state.json`` into the first job's dirs; ``extra_files``:
        {path: torch-serialisable object} written by the same thread (resume state)."""
        if self.busy():
            self.skipped += 1
            return False
        if jobs is None:
            jobs = [(out_dirs, self.flat.master if master is None else master)]
        # jobs whose source is the same buffer (a 1-client rank's global model IS its client
        # model) are copied and serialised once; the other dirs get a hard link to the file
        merged: List[tuple] = []
        by_src: Dict[Tuple[int, int], int] = {}
        for k, (dirs, src) in enumerate(jobs):
            key = (src.data_ptr(), src.numel())
            if key in by_src:
                merged[by_src[key]][0].extend((d, k == 0) for d in dirs)
            else:
                by_src[key] = len(merged)
                merged.append(([(d, k == 0) for d in dirs], src))
        jobs = merged
        bufs = [self._buf(i) for i in range(len(jobs))]
        if self.cuda:
            # snapshot on the device first (one D2D pass at HBM speed on the current stream), then
            # the D2H copies read the snapshot on the side stream: the training stream never waits
            # for PCIe (one-client round: the 438 MB D2H was 5.6 ms of device time per round on
            # the critical path). The next save reuses a snapshot only after this save's writer
            # thread has synchronised on `done` (busy() -> skipped / waited by the caller).
            cur = torch.cuda.current_stream(self.stream.device)
            while len(self.snaps) < len(jobs):
                self.snaps.append(torch.empty(self.flat.numel, dtype=torch.float32,
                                              device=self.stream.device))
            for snap, (_, src) in zip(self.snaps, jobs):
                snap.copy_(src)
            ev = cur.record_event()
            with torch.cuda.stream(self.stream):
                self.stream.wait_event(ev)
                for b, snap in zip(bufs, self.snaps):
                    b.copy_(snap, non_blocking=True)
                done = self.stream.record_event()
        else:
            for b, (_, src) in zip(bufs, jobs):
                b.copy_(src)
            done = None

        def _write():
            if done is not None:
                done.synchronize()
                # one snapshot stays for the next save; the extra ones of a multi-model save
                # (save_clients: one per hosted client) go back to the allocator now that their
                # D2H copies are done — not kept model-sized in HBM for the whole run
                del self.snaps[1:]
            st = state
            if st is not None and callable(st.get("_finalize")):
                # fields only known once device work queued before the save has finished (e.g. an
                # overlapped evaluation of this round): resolved here, on the writer thread
                st = dict(st)
                st.update(st.pop("_finalize")())
            for b, (dirs, _) in zip(bufs, jobs):
                host = b.numpy()
                first = None
                for d, with_state in dirs:
                    if first is None:
                        save_dir(d, self.model, host, self.layout, self.config, metadata)
                        first = d
                    else:
                        link_dir(first, d, self.config)
                    if st is not None and with_state:
                        with open(os.path.join(d, "state.json"), "w") as fh:
                            json.dump(st, fh, indent=2, sort_keys=True, default=str)
            for path, obj in (extra_files or {}).items():
                os.makedirs(os.path.dirname(path), exist_ok=True)
                torch.save(obj, path + ".tmp")
                os.replace(path + ".tmp", path)
            with self._lock:
                self.saved += 1
                self.last_dir = jobs[0][0][0][0] if jobs and jobs[0][0] else None

        if self.async_:
            self.future = self.pool.submit(_write)
        else:
            _write()
        return True

    def wait(self):
        if self.future is not None:
            self.future.result()
            self.future = None

    def close(self):
        self.wait()
        if self.pool:
            self.pool.shutdown(wait=True)


@torch.no_grad()
def load_into(model, flat, ckpt_dir: str, strict: bool = True) -> List[str]:
    """Load an HF-layout checkpoint (ours or transformers') into the flat master + params."""
    sd = read_safetensors(os.path.join(ckpt_dir, "model.safetensors"))
    items = model.adapter_items() if getattr(model, "lora", False) else model.hf_items()
    missing = []
    for name, get, set_ in items:
        if name in sd:
            set_(sd[name].to(get().device))
        else:
            missing.append(name)
    if strict and missing:
        raise KeyError(f"checkpoint missing {missing[:5]}")
    # params were written (compute dtype); refresh fp32 master from the exact fp32 file values
    if flat.master is not flat.param:
        lay = {n: (o, s) for n, o, s in hf_layout(model, flat)}
        for n, t in sd.items():
            if n in lay:
                o, s = lay[n]
                flat.master[o:o + t.numel()].copy_(t.reshape(-1).to(flat.master.device, torch.float32))
    return missing


def mirror_dir(src: str, dst: str):
    """Reference-compatible path (e.g. ./my_albert_model2) mirroring <out>/global."""
    if os.path.abspath(src) == os.path.abspath(dst):
        return
    os.makedirs(dst, exist_ok=True)
    for f in ("config.json", "model.safetensors"):
        s = os.path.join(src, f)
        if os.path.exists(s):
            shutil.copyfile(s, os.path.join(dst, f))
