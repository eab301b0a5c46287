import torch, sys
sys.path.insert(0, '.')
from dalgo.data.synthetic import blobs
from dalgo.models.kmeans import KMeans, KMeansConfig
n, d, k = 200_000, 128, 512
for noise in (1.0, 2.0, 4.0):
    X = blobs(n, d, k, device=torch.device('cuda'), dtype=torch.bfloat16, seed=13, noise=noise)
    km = KMeans(KMeansConfig(k=k, n_iterations=6, seed=3), X, 0, n)
    km.fit()
    print(noise, km.active_history, km.dense_history, flush=True)
