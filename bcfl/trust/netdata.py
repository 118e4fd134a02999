"""The reference's P2P network fixture.

10 nodes '0'..'9', all 90 ordered edges, edge weight = 1 / bandwidth_Mbps; the bandwidth table
below is transcribed from the ``G.add_edge(u, v, weight=1/bw)`` lines of
``All_graphs_IMDB_dataset.ipynb:73-167`` (identical in ``Medical_Transcriptions_All_graphs.ipynb``).
Markdown at ``Medical_Transcriptions_All_graphs.ipynb:983`` confirms ``weight(1,2)=1/145`` means a
145 Mbps channel. ``REF_BW_MBPS[u][v]`` is the u->v bandwidth (0 on the diagonal).
"""
import numpy as np

REF_BW_MBPS = np.array([
    [0, 259, 113, 479, 88, 400, 219, 209, 295, 135],
    [252, 0, 145, 343, 247, 421, 303, 383, 387, 272],
    [368, 232, 0, 308, 119, 309, 415, 435, 168, 361],
    [463, 128, 380, 0, 223, 490, 304, 370, 192, 338],
    [401, 479, 402, 465, 0, 285, 291, 370, 447, 205],
    [424, 382, 286, 340, 422, 0, 360, 224, 348, 153],
    [333, 434, 299, 363, 231, 408, 0, 486, 111, 234],
    [243, 426, 188, 180, 489, 192, 415, 0, 378, 148],
    [496, 299, 251, 343, 241, 475, 461, 434, 0, 435],
    [345, 126, 239, 196, 93, 237, 310, 370, 465, 0],
], dtype=np.float64)

# Recorded notebook outputs (golden values, All_graphs_IMDB_dataset.ipynb:52-54, :333, :489-491, :666)
REF_PAGERANK_THRESHOLDS = (0.08349251192983634, 0.11650748807016365)
REF_PAGERANK_ANOMALIES = [0, 4, 7, 9]
REF_MODZ_ANOMALIES = [8, 9]
REF_DBSCAN_ANOMALIES = []
REF_LOUVAIN_ANOMALIES = []

# Model sizes used by the reference's analytical info-passing numbers
BIOBERT_GB = 0.4036288568750024   # serverless_cancer_classification_with_BioBERT.ipynb:593
ALBERT_GB = 0.043                 # Medical_Transcriptions_All_graphs.ipynb:1096


def ref_weight_matrix() -> np.ndarray:
    """Directed weights 1/bw (nx.DiGraph of the notebook)."""
    W = np.zeros_like(REF_BW_MBPS)
    nz = REF_BW_MBPS > 0
    W[nz] = 1.0 / REF_BW_MBPS[nz]
    return W


def ref_undirected_weight_matrix() -> np.ndarray:
    """nx.Graph built from the same add_edge sequence: for u<v the later (v,u) line overwrites
    the (u,v) weight, so both directions carry 1/bw[v][u]."""
    W = ref_weight_matrix()
    U = np.zeros_like(W)
    n = W.shape[0]
    for u in range(n):
        for v in range(u + 1, n):
            U[u, v] = U[v, u] = W[v, u]
    return U
