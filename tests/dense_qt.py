"""Independent literal transcription of SpeedUp's qstep() algebra with dense 12x12 complex
numpy matrices — a second restatement used only to cross-check the C oracle's per-ion
quantum-trajectory step (test infrastructure; see oracle/mdqt_oracle.h for pinning status).

Every line follows /root/reference/laserCoolingPlusExpansionMDQTSpeedUp.cpp:
operators :1163-1215, qstep :438-717.  numpy's matmul orders sums its own way, so agreement
with the C oracle is at the 1e-14 level, not bitwise.
"""
import math

import numpy as np

r_D = 0.0617     # decayRatioD5Halves, SpeedUp:146
kRat = 0.395     # SpeedUp:147


def constants(density=2.0):
    gamToE = 174.07 / math.sqrt(density)                       # :79
    ratio = int(math.ceil(34.81 / math.sqrt(density)))          # :83
    dtQ = 0.002 / ratio                                         # :84
    pv2q = 1.1821 * density ** (1.0 / 6)                        # :85
    vKick = 0.001208 / pv2q                                     # :148
    return dict(gamToE=gamToE, ratio=ratio, dtQ=dtQ, pv2q=pv2q, vKick=vKick, vKickDP=vKick * kRat)


def operators(Om, OmDP):
    ident = np.eye(12)
    w = [ident[:, k].reshape(12, 1).astype(complex) for k in range(12)]   # wvFn1..12 -> w[0..11]
    H = lambda a: a.conj().T                                                # Armadillo .t()
    cs = [w[1] @ H(w[2]), w[1] @ H(w[3]), w[0] @ H(w[3]), w[0] @ H(w[4]), w[1] @ H(w[4]),
          w[0] @ H(w[5]), w[6] @ H(w[5]), w[7] @ H(w[5]), w[8] @ H(w[5]), w[7] @ H(w[4]),
          w[8] @ H(w[4]), w[9] @ H(w[4]), w[8] @ H(w[3]), w[9] @ H(w[3]), w[10] @ H(w[3]),
          w[9] @ H(w[2]), w[10] @ H(w[2]), w[11] @ H(w[2])]                 # :1163-1180
    r = r_D
    gs = [math.sqrt(1.), math.sqrt(2. / 3), math.sqrt(1. / 3), math.sqrt(2. / 3), math.sqrt(1. / 3),
          math.sqrt(1.), math.sqrt(r * 2. / 3), math.sqrt(r * 4. / 15), math.sqrt(r * 1. / 15),
          math.sqrt(r * 2. / 5), math.sqrt(r * 2. / 5), math.sqrt(r * 1. / 5), math.sqrt(r * 1. / 5),
          math.sqrt(r * 2. / 5), math.sqrt(r * 2. / 5), math.sqrt(r * 1. / 15), math.sqrt(r * 4. / 15),
          math.sqrt(r * 2. / 3)]                                           # :1181-1198
    hamDecay = np.zeros((12, 12), complex)
    decay = np.zeros((12, 12), complex)
    for j in range(18):                                                    # :1201-1204
        hamDecay = hamDecay - 1. / 2 * 1j * (gs[j] * gs[j] * H(cs[j]) @ cs[j])
        decay = decay + gs[j] * gs[j] * H(cs[j]) @ cs[j]
    coup = np.zeros((12, 12), complex)
    for k in range(6):                                                     # :1206-1210
        if k != 1 and k != 3:
            coup = coup + -1. * H(cs[k]) * gs[k] * Om / 2
    for k in range(6, 18):                                                 # :1211-1215
        if k not in (8, 11, 7, 10, 13, 16):
            coup = coup + -1. * H(cs[k]) * gs[k] * OmDP / 2 / math.sqrt(r)
    return dict(w=w, cs=cs, gs=gs, hamDecay=hamDecay, decay=decay, coup=coup)


def qstep_ion(psi, vx, tPart, t, u, p):
    """One ion through qstep (:478-705).  psi: complex[12]; u: uniforms u1..u5.
    p: dict with Om, OmDP, detuning, detuningDP, fracOfSig, Te, density, sig0.
    Returns (psi', vx', tPart', jumped)."""
    c = constants(p["density"])
    ops = operators(p["Om"], p["OmDP"])
    w, gs, decay = ops["w"], ops["gs"], ops["decay"]
    H = lambda a: a.conj().T
    dtQuant, gamToE = c["dtQ"], c["gamToE"]
    expDet = 0.0126 * p["fracOfSig"] * p["Te"] * t / (
        math.sqrt(p["density"]) * p["sig0"] * math.sqrt(1 + 0.00014314 * t * t * p["Te"] / (p["density"] * p["sig0"] * p["sig0"])))
    wvFn = np.asarray(psi, complex).reshape(12, 1)
    velQuant = vx * c["pv2q"]
    tPart = tPart + dtQuant
    dp = (dtQuant * gamToE * H(wvFn) @ decay @ wvFn)[0, 0].real
    ui = iter(u)
    rand = next(ui)
    det, detDP, Om, OmDP = p["detuning"], p["detuningDP"], p["Om"], p["OmDP"]
    if rand > dp:
        rho = wvFn @ H(wvFn)
        pim = lambda a, b: (H(w[a - 1]) @ rho @ w[b - 1])[0, 0].imag
        kick = (1 * c["vKick"] * Om * (pim(2, 3) * gs[0] + pim(1, 4) * gs[2] - pim(2, 5) * gs[4] - pim(1, 6) * gs[5])
                * dtQuant * gamToE
                + c["vKickDP"] * (OmDP / r_D) * (pim(9, 6) * gs[8] + pim(10, 5) * gs[11] + pim(11, 4) * gs[14]
                                                 + pim(12, 3) * gs[17] - pim(7, 6) * gs[6] - pim(8, 5) * gs[9]
                                                 - pim(9, 4) * gs[12] - pim(10, 3) * gs[15]) * dtQuant * gamToE)
        dR = -det - velQuant - expDet
        dL = -det + velQuant + expDet
        ph = np.exp(1j * 2. * (velQuant + expDet) * (1 + kRat) * tPart * gamToE)
        hamC = (ops["coup"] - OmDP / 2 * w[8] @ H(w[5]) * gs[8] / math.sqrt(r_D) * ph
                - OmDP / 2 * w[9] @ H(w[4]) * gs[11] / math.sqrt(r_D) * ph)
        hP = dR * (w[2] @ H(w[2]) + w[3] @ H(w[3])) + dL * (w[4] @ H(w[4]) + w[5] @ H(w[5]))
        hD = ((-det + detDP + (1 - kRat) * (velQuant + expDet)) * (w[6] @ H(w[6]) + w[7] @ H(w[7]))
              + (-det + detDP + (kRat - 1) * (velQuant + expDet)) * (w[10] @ H(w[10]) + w[11] @ H(w[11]))
              + (-det + detDP - velQuant - expDet - kRat * (velQuant + expDet)) * (w[8] @ H(w[8]) + w[9] @ H(w[9])))
        hamil = (hP + hD) + hamC + H(hamC) + ops["hamDecay"]
        dtHalf = dtQuant * gamToE / 2
        M = np.eye(12) - 1j * dtQuant * gamToE * hamil
        hh = dtQuant * gamToE

        def stage(y):
            dpy = (hh * H(y) @ decay @ y)[0, 0].real
            pref = 1 / math.sqrt(1 - dpy)
            return 1. / hh * (pref * M @ y - y)

        k1 = stage(wvFn); y1 = wvFn + dtHalf * k1
        k2 = stage(y1); y2 = wvFn + dtHalf * k2
        k3 = stage(y2); y3 = wvFn + hh * k3
        k4 = stage(y3)
        wvFn = wvFn + (k1 + 3 * k2 + 3 * k3 + k4) / 8 * hh
        jumped = False
    else:
        jumped = True
        tPart = 0.0
        rand2 = next(ui)
        n = [abs(wvFn[k, 0]) ** 2 for k in (2, 3, 4, 5)]
        tot = n[0] + n[1] + n[2] + n[3]
        prob3, prob4, prob5 = n[0] / tot, n[1] / tot, n[2] / tot
        wvFn = np.zeros((12, 1), complex)
        randDOrS = next(ui)
        randDir = next(ui)
        sDecay = not (randDOrS < r_D / (r_D + 1))
        if sDecay:
            kick = c["vKick"] if randDir < 0.5 else -c["vKick"]
        else:
            kick = c["vKickDP"] if randDir < 0.5 else -c["vKickDP"]
        g2 = lambda k: gs[k] * gs[k] / r_D
        if rand2 < prob3:
            if sDecay:
                tgt = 1
            else:
                u3 = next(ui)
                tgt = 11 if u3 < g2(17) else (10 if u3 < g2(17) + g2(16) else 9)
        elif rand2 < prob3 + prob4:
            u3 = next(ui)
            if sDecay:
                tgt = 0 if u3 < gs[2] * gs[2] else 1
            else:
                tgt = 10 if u3 < g2(14) else (9 if u3 < g2(14) + g2(13) else 8)
        elif rand2 < prob3 + prob4 + prob5:
            u3 = next(ui)
            if sDecay:
                tgt = 1 if u3 < gs[4] * gs[4] else 0
            else:
                tgt = 9 if u3 < g2(11) else (8 if u3 < g2(11) + g2(10) else 7)
        else:
            if sDecay:
                tgt = 0
            else:
                u3 = next(ui)
                tgt = 8 if u3 < g2(8) else (7 if u3 < g2(8) + g2(7) else 6)
        wvFn[tgt, 0] = 1.0
    return wvFn.reshape(12), vx + kick, tPart, jumped
