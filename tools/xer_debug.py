import sys
import numpy as np
import scipy.sparse as sp
sys.path.insert(0, "gnn-sparsification-research_amd")
sys.path.insert(0, "tests")
from conftest import load_golden  # noqa: E402
import gsparse  # noqa: E402
g = load_golden(sys.argv[1] if len(sys.argv) > 1 else "roman2000")
n = int(g["num_nodes"])
adj = sp.csr_matrix((g["data"], g["indices"], g["indptr"]), shape=(n, n))
try:
    er = gsparse.calculate_effective_resistance_scores(adj)
    print("er", er[:4], "min", er.min(), "max", er.max())
except Exception as e:
    print("ERR", e)
