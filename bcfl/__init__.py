"""bcfl — MI355X-native decentralized federated fine-tuning.

Capabilities follow the reference research scripts (Flower FedAvg "server" case and the
hand-written "serverless" averaging case, see ``/root/reference/src``) plus the features the
reference only describes (async P2P gossip, blockchain ledger, PageRank anomaly filtering,
information-passing-time model; ``README.md:10`` of the reference).

Layout::

    bcfl.config    dataclass config, per-script presets, CLI
    bcfl.data      synthetic IMDB-shaped datasets, partitioners, packed (varlen) batching
    bcfl.models    BERT / ALBERT / DistilBERT / Llama(+LoRA) with HF state-dict names
    bcfl.ops       autograd ops bound to hand-written HIP/CDNA4 kernels (bcfl._C)
    bcfl.parallel  process groups, flat parameter buffers, FedAvg all-reduce, P2P gossip
    bcfl.fl        Client, ServerFedAvg, ServerlessGossip, anomaly filter, virtual clients
    bcfl.trust     native PageRank / modified-Z / DBSCAN / path model, blockchain ledger
    bcfl.ckpt      safetensors checkpoints (HF layout), async writer, resume
    bcfl.utils     timers, metrics JSONL, reference-compatible telemetry prints
"""

__version__ = "0.1.0"

import os as _os

# Client lanes run several training steps concurrently on separate HIP streams. hipBLASLt's
# Stream-K GEMM kernels (SK3) spin-wait on partial tiles produced by other workgroups of the SAME
# launch; two of them running at once can each hold the CUs the other one's producers need and
# deadlock (observed: Llama-3-8B LoRA, 2 lanes, GPU 100 % busy, zero memory traffic, forever).
# Data-parallel Stream-K mode computes whole tiles per workgroup (no cross-workgroup waits).
# Must be set before the first GEMM initialises the Tensile library.
_os.environ.setdefault("TENSILE_STREAMK_DATA_PARALLEL", "1")
