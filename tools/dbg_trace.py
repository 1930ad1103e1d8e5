import sys, os, ctypes as C, numpy as np, torch
sys.path.insert(0, 'mahi-mpc_amd'); sys.path.insert(0, 'tests')
import mmpc, oracle_lib as o
d = np.load('tools/debug/cfg2_nonconverged.npz')
path = mmpc.write_model_json('/tmp/m.json', 'nonlinear_double_pendulum', 4, 2, 2000, 30)
s = mmpc.Solver(path)
L = mmpc.lib()
L.mmpc_debug_solve_trace.argtypes = [C.c_void_p, C.c_int64] + [C.c_void_p] * 4 + [C.c_int64] + [C.c_void_p] * 6
B = len(d['idx'])
t = lambda a: torch.tensor(np.ascontiguousarray(a), dtype=torch.float64, device='cuda')
x0, up, tr = t(d['x0']), t(d['u_prev']), t(d['traj'])
w = t([10, 1, 5, 5, 5, 5, .01, .01])
V = torch.zeros((B, s.NV), dtype=torch.float64, device='cuda')
st = torch.zeros(B, dtype=torch.int32, device='cuda'); it = torch.zeros(B, dtype=torch.int32, device='cuda')
kk = torch.zeros(B, dtype=torch.float64, device='cuda'); trc = torch.zeros((B, 51, 8), dtype=torch.float64, device='cuda')
rc = L.mmpc_debug_solve_trace(s._h, B, x0.data_ptr(), up.data_ptr(), tr.data_ptr(), w.data_ptr(), 0, V.data_ptr(),
                              st.data_ptr(), it.data_ptr(), kk.data_ptr(), trc.data_ptr(), None)
torch.cuda.synchronize()
print('rc', rc, 'status', st.cpu().numpy(), 'iters', it.cpu().numpy())
np.set_printoptions(linewidth=200, precision=3)
for b in range(B):
    T = trc[b].cpu().numpy()
    for i in range(min(int(it[b]) + 1, 51)):
        print(i, ' '.join('%.3e' % v for v in T[i]))
r = o.solve_batch(30, 0.002, d['x0'], d['u_prev'], d['traj'], np.array([10, 1, 5, 5, 5, 5, .01, .01]))
print('oracle', r['status'], r['iters'], r['kkt'])
Vg = V.cpu().numpy()
print('V rel diff', np.abs(Vg - r['V']).max() / np.abs(r['V']).max())
