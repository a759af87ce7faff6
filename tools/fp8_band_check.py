import numpy as np, torch, sys, time
sys.path.insert(0, '/root/repo')
import bench
torch.set_num_threads(8)
cfg = bench.CONFIGS[3]
cent = bench.make_centres(torch, cfg, 'cpu', 3)
N = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
xq = bench.gen_queries(torch, cfg, cent, 32, 'cpu', 3).numpy().astype(np.float64)
D = xq.shape[1]
def e4m3(v):
    a = np.abs(v); e = np.floor(np.log2(np.maximum(a, 1e-30))); e = np.maximum(e, -6)
    qn = 2.0 ** (e - 3); r = np.rint(v / qn) * qn
    return np.clip(r, -448, 448)
def mx(x, B=32):
    n = x.shape[0]; Dp = (D + B - 1)//B*B
    xp = np.zeros((n, Dp)); xp[:, :D] = x
    b2 = xp.reshape(n, Dp//B, B)
    amax = np.abs(b2).max(-1, keepdims=True)
    sc = 2.0 ** (np.floor(np.log2(np.maximum(amax, 1e-30))) - 8)
    return (e4m3(b2 / sc) * sc).reshape(n, Dp)[:, :D]
def i8(x, B=64):
    n = x.shape[0]; Dp = (D + B - 1)//B*B
    xp = np.zeros((n, Dp)); xp[:, :D] = x
    b2 = xp.reshape(n, Dp//B, B)
    s = np.abs(b2).max(-1, keepdims=True) / 127.0; s[s == 0] = 1
    return (np.rint(b2 / s) * s).reshape(n, Dp)[:, :D]
def seg(x, bounds=(0, 48, 176, 1968)):
    """int8 with one scale per concat part (colour 48 | SIFT 128 | DreamSim 1792)"""
    out = np.empty_like(x)
    for a, b in zip(bounds[:-1], bounds[1:]):
        s = np.abs(x[:, a:b]).max(1, keepdims=True) / 127.0; s[s == 0] = 1
        out[:, a:b] = np.rint(x[:, a:b] / s) * s
    return out
def bf16(x):
    return torch.from_numpy(x.astype(np.float32)).bfloat16().double().numpy()
variants = {"bf16": bf16, "i8b64": i8, "mxfp8": mx, "i8seg": seg}
qv = {"bf16": bf16(xq), "i8b64": xq, "mxfp8": mx(xq), "mxfp8_qexact": xq, "i8seg": seg(xq),
      "i8seg_qexact": xq}
rowv = {"bf16": "bf16", "i8b64": "i8b64", "mxfp8": "mxfp8", "mxfp8_qexact": "mxfp8", "i8seg": "i8seg",
        "i8seg_qexact": "i8seg"}
AP = {v: [] for v in qv}; RR = {v: [] for v in variants}
for blk in bench.gen_rows(torch, cfg, cent, 0, N, 'cpu', 3):
    xb = blk.numpy().astype(np.float64)
    deqs = {v: f(xb) for v, f in variants.items()}
    for v in variants: RR[v].append(np.linalg.norm(xb - deqs[v], axis=1))
    for v, q in qv.items():
        dq = deqs[rowv[v]]
        AP[v].append((xq**2).sum(1)[:, None] + (xb**2).sum(1)[None] - 2 * q @ dq.T)
k = 10
for v in qv:
    ap = np.concatenate(AP[v], 1); r = np.concatenate(RR[rowv[v]]); R = r.max()
    dqn = np.linalg.norm(xq - qv[v], axis=1)
    idx = np.argsort(ap, 1)[:, :k]
    T = np.take_along_axis(ap, idx[:, k-1:k], 1)[:, 0]
    xn = 1.0 * np.sqrt(4.0)   # |x~| ~ 2 (four unit-norm parts? concat of 3) upper
    e = 2 * (np.linalg.norm(xq, axis=1) * R + dqn * (2.0 + R))
    band = (ap <= (T + 2 * e)[:, None]).sum(1)
    print(v, "R %.4f dq %.4f | band median %d p90 %d max %d" % (R, dqn.max(), np.median(band), np.percentile(band, 90), band.max()), flush=True)
