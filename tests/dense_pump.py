"""Independent literal transcription of the optical-pumping qstep() of the spin-tagging
programs with dense complex numpy matrices — a second restatement used only to cross-check the
C oracle (test infrastructure; see oracle/mdqt_oracle.h for the pinning status).

Follows /root/reference/randomFrozenStartTag408Linear.cpp (qstep :396-598, cs/gs in main
:1000-1019), randomFrozenStartTag408Quad.cpp (coupling :97 of its qstep) and
randomFrozenStartTag422Linear.cpp (qstep :390-566, cs/gs in main).  Models: 1 = 408 linear,
2 = 408 quad, 3 = 422 linear; psi is padded to the engine's 12-state layout.
"""
import math

import numpy as np



def model_constants(model, density=2.0):
    """the pumping programs' constants: randomFrozenStartTag408Linear.cpp:67-75, :118 (408Quad
    :69-77, :121) and randomFrozenStartTag422Linear.cpp:66-74, :116 (C round(): half away from 0)"""
    if model == 3:
        gamToE = 174.07 * .894 / math.sqrt(density)
        ratio = int(math.floor(34.81 * .894 / math.sqrt(density) + 0.5))
        pv2q = 1.1821 * density ** (1.0 / 6) * .967
        decay = 0.0754
    else:
        gamToE = 174.07 / math.sqrt(density)
        ratio = int(math.floor(34.81 / math.sqrt(density) + 0.5))
        pv2q = 1.1821 * density ** (1.0 / 6)
        decay = 0.0617
    return dict(gamToE=gamToE, ratio=ratio, dtQ=0.002 / ratio, pv2q=pv2q, decayRatio=decay)


def operators(model, decayRatio):
    n = 5 if model == 3 else 7
    ident = np.eye(n)
    w = [ident[:, k].reshape(n, 1).astype(complex) for k in range(n)]   # wvFn1.. -> w[0..]
    H = lambda a: a.conj().T
    if model == 3:
        cs = [w[1] @ H(w[2]), w[1] @ H(w[3]), w[0] @ H(w[3]), w[0] @ H(w[2]), w[4] @ H(w[2]), w[4] @ H(w[3])]
        gs = [2. / 3, 1. / 3, 2. / 3, 1. / 3, decayRatio, decayRatio]
    else:
        cs = [w[0] @ H(w[2]), w[0] @ H(w[3]), w[0] @ H(w[4]), w[1] @ H(w[3]), w[1] @ H(w[4]), w[1] @ H(w[5]),
              w[6] @ H(w[2]), w[6] @ H(w[3]), w[6] @ H(w[4]), w[6] @ H(w[5])]
        gs = [1, 2. / 3, 1. / 3, 1. / 3, 2. / 3, 1, decayRatio, decayRatio, decayRatio, decayRatio]
    return n, w, cs, gs


def qstep_ion(psi12, vx, tPart, u, model, Om, detuning, density=2.0):
    """One ion through the pumping qstep; u: the uniforms in the reference's draw order.
    Returns (psi12', vx', tPart', jumped)."""
    c = model_constants(model, density)
    decayRatio = c["decayRatio"]
    n, w, cs, gs = operators(model, decayRatio)
    H = lambda a: a.conj().T
    dtQuant, gamToE = c["dtQ"], c["gamToE"]
    hh = dtQuant * gamToE
    wvFn = np.asarray(psi12, complex)[:n].reshape(n, 1)
    velQuant = vx * c["pv2q"]
    tPart = tPart + dtQuant
    nch = len(cs)

    def dp_of(y):
        d = 0.0
        for j in range(nch):
            d = d + (hh * H(y) @ H(cs[j]) @ cs[j] @ y)[0, 0] * gs[j]
        return d.real

    dp = dp_of(wvFn)
    ui = iter(u)
    rand = next(ui)
    if rand > dp:
        dR = -detuning - velQuant
        dL = -detuning + velQuant
        if model == 1:
            C = (-Om / 2 * w[1] @ H(w[3]) * math.sqrt(gs[3]) - Om / 2 * w[1] @ H(w[5]) * math.sqrt(gs[5])
                 - Om / 2 * w[0] @ H(w[2]) * math.sqrt(gs[0]) - Om / 2 * w[0] @ H(w[4]) * math.sqrt(gs[2]))
            E = dR * (w[2] @ H(w[2]) + w[3] @ H(w[3])) + dL * (w[4] @ H(w[4]) + w[5] @ H(w[5]))
        elif model == 2:
            C = -Om / 2 * w[1] @ H(w[5]) * math.sqrt(gs[5]) - Om / 2 * w[0] @ H(w[4]) * math.sqrt(gs[2])
            E = dR * (w[2] @ H(w[2]) + w[3] @ H(w[3])) + dL * (w[4] @ H(w[4]) + w[5] @ H(w[5]))
        else:
            C = -Om / 2 * w[1] @ H(w[2]) * math.sqrt(gs[0]) - Om / 2 * w[0] @ H(w[3]) * math.sqrt(gs[2])
            E = dR * (w[2] @ H(w[2])) + dL * (w[3] @ H(w[3]))
        hamDecay = np.zeros((n, n), complex)
        for j in range(nch):
            hamDecay = hamDecay - 1. / 2 * 1j * (gs[j] * H(cs[j]) @ cs[j])
        hamil = E + C + H(C) + hamDecay
        M = np.eye(n) - 1j * hh * hamil

        def stage(y):
            pref = 1 / math.sqrt(1 - dp_of(y))
            return 1. / hh * (pref * M @ y - y)

        k1 = stage(wvFn); y1 = wvFn + hh / 2 * k1
        k2 = stage(y1); y2 = wvFn + hh / 2 * k2
        k3 = stage(y2); y3 = wvFn + hh * k3
        k4 = stage(y3)
        wvFn = wvFn + (k1 + 3 * k2 + 3 * k3 + k4) / 8 * hh
        jumped = False
    else:
        jumped = True
        tPart = 0.0
        rand2 = next(ui)
        nr = [abs(wvFn[k, 0]) ** 2 for k in range(2, 6 if model != 3 else 4)]
        randDOrS = next(ui)
        sDecay = not (randDOrS < decayRatio / (decayRatio + 1))
        if model == 3:
            prob3 = nr[0] / (nr[0] + nr[1])
            if rand2 < prob3:
                tgt = (1 if next(ui) < gs[0] else 0) if sDecay else 4
            else:
                tgt = (0 if next(ui) < gs[2] else 1) if sDecay else 4
        else:
            tot = nr[0] + nr[1] + nr[2] + nr[3]
            prob3, prob4, prob5 = nr[0] / tot, nr[1] / tot, nr[2] / tot
            next(ui)                                    # randDir (drawn, unused)
            if rand2 < prob3:
                tgt = 0 if sDecay else 6
            elif rand2 < prob3 + prob4:
                tgt = (0 if next(ui) < gs[1] else 1) if sDecay else 6
            elif rand2 < prob3 + prob4 + prob5:
                tgt = (0 if next(ui) < gs[2] else 1) if sDecay else 6
            else:
                tgt = 1 if sDecay else 6
        wvFn = np.zeros((n, 1), complex)
        wvFn[tgt, 0] = 1.0
    out = np.zeros(12, complex)
    out[:n] = wvFn.reshape(n)
    return out, vx, tPart, jumped
