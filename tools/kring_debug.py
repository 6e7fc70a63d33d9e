"""Debug helper: device kRing / kLoop lists vs the oracle on the global res-r cells of
test_h3_kring_kloop_equal_oracle; for each mismatch, whether the oracle took the
fallback and whether the cell alone gives the right list."""
import sys, os, numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, ROOT + '/oracle')
import mosaic_amd as M, oracle as O
g = torch.device('cuda', 0)
L = O._h3_kring_lib()
for res in (2, 3):
    rng = np.random.default_rng(900 + res)
    lon = rng.uniform(-180, 180, 600); lat = np.degrees(np.arcsin(rng.uniform(-1, 1, 600)))
    cells = O.h3_points_to_cells(lon, lat, res).astype(np.int64)
    for k in (1, 2):
        ids, off = M.grid_cellkring(torch.from_numpy(cells).to(g), k, M.H3IndexSystem())
        ids, off = ids.cpu().numpy(), off.cpu().numpy()
        bad = [i for i, c in enumerate(cells) if [int(v) for v in ids[off[i]:off[i + 1]]] != O.h3_k_ring(int(c), k)]
        info = []
        for i in bad[:6]:
            buf = np.zeros(L.orc_h3_max_kring_size(k), dtype=np.uint64)
            fb = L.orc_h3_kring_raw(int(cells[i]), k, O._ptr(buf, O._u64p))
            a, o2 = M.grid_cellkring(torch.from_numpy(cells[i:i + 1]).to(g), k, M.H3IndexSystem())
            alone = [int(v) for v in a.cpu().numpy()] == O.h3_k_ring(int(cells[i]), k)
            got = [int(v) for v in ids[off[i]:off[i + 1]]]
            ref = O.h3_k_ring(int(cells[i]), k)
            tab = [0] * len(buf)
            for c in ref:
                q = c % len(buf)
                while tab[q]:
                    q = (q + 1) % len(buf)
                tab[q] = c
            info.append((i, hex(int(cells[i])), "oracle_fallback=%d" % fb, "alone_ok=%s" % alone,
                         "same set %s" % (sorted(got) == sorted(ref)), "hash order %s" % (got == [c for c in tab if c])))
        print("res", res, "k", k, "bad", len(bad), info, flush=True)
