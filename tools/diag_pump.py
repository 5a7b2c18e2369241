"""GPU diagnostic: per-ion divergence of the pumping-model trajectories vs the oracle."""
import sys
import numpy as np
sys.path.insert(0, ".")
import mdqtplasmasims_amd as M
from oracle import oracle as O

model = int(sys.argv[1]) if len(sys.argv) > 1 else 1
kw = dict(Om=0.7, detuning=-2.5, qt_model=model, N0=400, seed=5, rng_mode=1)
o = O.OracleSim(nthreads=4, **kw).init()
st = o.get_state()
n = 5 if model == 3 else 7
rng = np.random.default_rng(model)
z = np.zeros((st["psi"].shape[0], 12), complex)
z[:, :n] = rng.normal(size=(z.shape[0], n)) + 1j * rng.normal(size=(z.shape[0], n))
z /= np.linalg.norm(z, axis=1, keepdims=True)
psi = np.stack([z.real, z.imag], -1)
s = M.Simulation(**kw)
for x in (s, o):
    x.set_state(st["R"], st["V"], psi, st["tPart"], 0.0)
for step in range(75):
    if step % 25 == 0:
        s.forces(); o.forces()
        Fa, Fb = s.get_state()["F"], o.get_state()["F"]
        print("forces rel diff", np.abs(Fa - Fb).max() / np.abs(Fb).max())
    s.step(); o.step()
    s.qstep(); o.qstep()
    a, b = s.get_state(), o.get_state()
    d = np.abs(a["psi"] - b["psi"]).max(axis=(1, 2))
    i = int(np.argmax(d))
    if step == 0:
        dRa = np.abs(a["R"] - b["R"])
        c, j = np.unravel_index(np.argmax(dRa), dRa.shape)
        print("dR ion", j, "coord", c, "gpu", repr(a["R"][c, j]), "orc", repr(b["R"][c, j]),
              "R0", repr(st["R"][c, j]), "V", repr(a["V"][c, j]), repr(b["V"][c, j]), "L", o.const("L"), s.const("L"))
    if d[i] > 1e-12 or step % 10 == 0:
        print(step, "maxdiff", d[i], "ion", i, "tPart gpu/orc", a["tPart"][i], b["tPart"][i],
              "dV", np.abs(a["V"] - b["V"]).max(), "dR", np.abs(a["R"] - b["R"]).max())
        print("   gpu", np.round(a["psi"][i, :n], 6).tolist())
        print("   orc", np.round(b["psi"][i, :n], 6).tolist())
    if d[i] > 1e-9:
        break
