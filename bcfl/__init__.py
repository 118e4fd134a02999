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
