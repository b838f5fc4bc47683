"""Exact effective-resistance golden vectors (metrics.py:124-175) for the
medium fixtures, made by RUNNING the reference function in the build
container (it needs /root/reference):

    OPENBLAS_NUM_THREADS=1 python tests/golden/make_golden_exact_er.py

Input: the canonical CSR already stored in each fixture; output:
``exact_er_<name>.npz`` with the reference's scores (CSR order).
"""

from __future__ import annotations

import os
import sys
import time

import numpy as np
import scipy.sparse as sp

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, "/root/reference/src/sparsification")

import metrics  # noqa: E402  (the reference module, imported by path)

for name in ["rmat10", "roman2000", "cora_like", "directed_dup"]:
    g = np.load(os.path.join(HERE, f"{name}.npz"))
    n = int(g["num_nodes"])
    adj = sp.csr_matrix((g["data"], g["indices"], g["indptr"]), shape=(n, n))
    if (adj != adj.T).nnz:
        print(f"{name}: not symmetric, skipped")
        continue
    t0 = time.time()
    er = metrics.calculate_effective_resistance_scores(adj)
    np.savez_compressed(os.path.join(HERE, f"exact_er_{name}.npz"), scores_effective_resistance=er)
    print(f"{name}: n={n} nnz={adj.nnz} {time.time() - t0:.1f}s", flush=True)
