import sys, os; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import time, numpy as np, torch
print("torch", torch.__version__, torch.cuda.is_available(), torch.cuda.get_device_name(0))
from image_recommender_amd import faiss_compat as faiss, _lib
print(_lib.load().knn_version())
xb = np.random.default_rng(0).standard_normal((10000, 512)).astype(np.float32)
idx = faiss.IndexFlatL2(512); idx.add(xb)
D, I = idx.search(xb[:5], 5); print(D, I)
