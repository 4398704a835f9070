#!/usr/bin/env python3
"""Exhaustive check of k_t1_cm3's v_bitop3 context formulas (t1.hip
zc_masks / sc_masks) against the case-by-case forms of ISO 15444-1 Tables
D.1-D.3 as the previous kernel wrote them, on all 256 neighbourhoods of each
band.  bitop3 table convention: bit (a << 2 | b << 1 | c) of TT = f(a, b, c)."""
import itertools


def b3(a, b, c, tt):
    return (tt >> ((a << 2) | (b << 1) | c)) & 1


def N(x):
    return 1 - x


def zc_table(UL, U, UR, L, R, DL, D, DR, band):
    s1x, s1a, s2x, s2a = UL ^ UR, UL & UR, DL ^ DR, DL & DR
    dge1, dge2 = s1x | s1a | s2x | s2a, s1a | s2a | (s1x & s2x)
    if band == 3:
        dge3 = (s1a & (s2x | s2a)) | (s2a & (s1x | s1a))
        hvge1 = L | R | U | D
        hvge2 = (L & R) | (U & D) | ((L ^ R) & (U ^ D))
        hv1 = hvge1 & N(hvge2)
        d2, d1, d0 = dge2 & N(dge3), dge1 & N(dge2), N(dge1)
        I = [0, d0 & hv1, d0 & hvge2, d1 & N(hvge1), d1 & hv1, d1 & hvge2, d2 & N(hvge1), d2 & hvge1, dge3]
    else:
        A1, A2 = (U, D) if band == 1 else (L, R)
        B1, B2 = (L, R) if band == 1 else (U, D)
        h2, h1, h0 = A1 & A2, A1 ^ A2, N(A1 | A2)
        vge1, v2, v1 = B1 | B2, B1 & B2, B1 ^ B2
        nv = N(vge1)
        I = [0, h0 & nv & dge1 & N(dge2), h0 & nv & dge2, h0 & v1, h0 & v2, h1 & nv & N(dge1), h1 & nv & dge1,
             h1 & vge1, h2]
    return (I[1] | I[3] | I[5] | I[7], I[2] | I[3] | I[6] | I[7], I[4] | I[5] | I[6] | I[7], I[8])


def zc_bitop3(UL, U, UR, L, R, DL, D, DR, band):
    u, d = UL | UR, DL | DR
    dge1, s2a = u | d, DL & DR
    dge2 = b3(u, d, b3(UL, UR, s2a, 0xEA), 0xEA)
    if band == 3:
        dge3 = b3(s2a, u, UL & UR & d, 0xEA)
        a, c = L | R, U | D
        hvge1 = a | c
        hvge2 = b3(a, c, b3(L, R, U & D, 0xEA), 0xEA)
        d2, d1 = b3(dge2, dge3, dge3, 0x30), b3(dge1, dge2, dge2, 0x30)
        hv1 = b3(hvge1, hvge2, hvge2, 0x30)
        return (b3(d2, hvge1, b3(d1, dge1, hv1, 0x72), 0xEA), b3(dge1, hvge2, b3(d1, hvge1, d2, 0xBA), 0xAE),
                b3(d1, hvge1, d2, 0xEA), dge3)
    A1, A2 = (U, D) if band == 1 else (L, R)
    B1, B2 = (L, R) if band == 1 else (U, D)
    e, x = b3(dge1, dge2, dge2, 0x30), A1 ^ A2
    return (b3(x, b3(B1, B2, dge1, 0xFD), b3(A1, A2, b3(B1, B2, e, 0x3E), 0x02), 0xEA),
            b3(x, B1 | B2 | dge1, b3(A1, A2, b3(B1, B2, dge2, 0x3E), 0x02), 0xEA),
            b3(A1, A2, B1 & B2, 0x3E), A1 & A2)


def sc_table(Ls, Ln, Rs, Rn, Us, Un, Ds, Dn):
    pL, nL, pR, nR = Ls & N(Ln), Ls & Ln, Rs & N(Rn), Rs & Rn
    pU, nU, pD, nD = Us & N(Un), Us & Un, Ds & N(Dn), Ds & Dn
    hp, hn = (pL & pR) | ((pL | pR) & N(nL | nR)), (nL & nR) | ((nL | nR) & N(pL | pR))
    vp, vn = (pU & pD) | ((pU | pD) & N(nU | nD)), (nU & nD) | ((nU | nD) & N(pU | pD))
    hz, vz = N(hp | hn), N(vp | vn)
    I13, I12, I11 = (hp & vp) | (hn & vn), (hp | hn) & vz, (hp & vn) | (hn & vp)
    I9, I10 = hz & vz, hz & (vp | vn)
    return (I9 | I11 | I13, I10 | I11, I12 | I13, hn | (hz & vn))


def sc_bitop3(Ls, Ln, Rs, Rn, Us, Un, Ds, Dn):
    def pair(As, An, Bs, Bn):
        nA, nB = As & An, Bs & Bn
        pA, pB = b3(As, An, An, 0x30), b3(Bs, Bn, Bn, 0x30)
        return b3(pB, nA, b3(As, An, nB, 0x10), 0xBA), b3(nB, pA, b3(nA, pB, pB, 0x30), 0xBA)
    hp, hn = pair(Ls, Ln, Rs, Rn)
    vp, vn = pair(Us, Un, Ds, Dn)
    hnz, vnz = hp | hn, vp | vn
    opp = b3(hn, vp, hp & vn, 0xEA)
    return (N(hnz ^ vnz), b3(hnz, vnz, opp, 0xAE), b3(hnz, opp, opp, 0x30), b3(hn, hnz, vn, 0xF2))


if __name__ == "__main__":
    cases = list(itertools.product((0, 1), repeat=8))
    bad = sum(zc_table(*c, band) != zc_bitop3(*c, band) for band in range(4) for c in cases)
    bad += sum(sc_table(*c) != sc_bitop3(*c) for c in cases)
    print("mismatches:", bad)
    raise SystemExit(1 if bad else 0)
