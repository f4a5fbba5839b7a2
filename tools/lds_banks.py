"""Bank-conflict check of the LDS fragment reads against the CDNA4 lane groups
(MI355X_MICROARCH.md, LDS table): cycles per wave-instruction vs the conflict-free count."""
B128 = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
        list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
B128 += [[l + 32 for l in g] for g in B128]
B64 = [list(range(32)), list(range(32, 64))]


def cycles(addr, groups, width):
    tot = 0
    for g in groups:
        banks = {}
        for l in g:
            a = addr(l)
            for w in range(width // 4):
                b = (a // 4 + w) % 64
                banks.setdefault(b, set()).add((a // 4 + w) // 64)
        tot += max(len(v) for v in banks.values())
    return tot


def ring_kc(lane, f0=0):          # g3_frag<true>: 64-B rows
    r = f0 + (lane & 15)
    slot = (lane >> 4) ^ ((r >> 2) & 3)
    return r * 64 + slot * 16


def pair_kc(lane, f0=0, u=0):     # g3p_frag<true>: 128-B rows
    r = f0 + (lane & 15)
    slot = (u * 4 + (lane >> 4)) ^ ((r >> 1) & 7)
    return r * 128 + slot * 16


def gru_ring(lane, uu=0):         # ring_core: 256-B rows
    r = lane & 15
    return r * 256 + (((uu * 4 + (lane >> 4)) ^ (r & 15)) * 16)


def tr(lane, f0=0, half=0):       # g3_frag<false>: ds_read_b64_tr_b16
    h, q, p = lane >> 4, (lane & 15) >> 2, lane & 3
    j = (f0 >> 2) + p
    kr = 8 * h + q + 4 * half
    s = (j >> 1) ^ (2 * (kr & 3) + 8 * ((kr >> 3) & 1))
    return kr * 512 + s * 16 + (j & 1) * 8


if __name__ == '__main__':
    print('ring KC  b128:', [cycles(lambda l: ring_kc(l, f0), B128, 16) for f0 in (0, 16, 32)], '(ideal 4)')
    print('pair KC  b128:', [cycles(lambda l: pair_kc(l, f0, u), B128, 16) for f0 in (0, 16) for u in (0, 1)], '(ideal 4)')
    print('gru ring b128:', [cycles(lambda l: gru_ring(l, uu), B128, 16) for uu in range(4)], '(ideal 4)')
    print('tr b64       :', [cycles(lambda l: tr(l, f0, hf), B64, 8) for f0 in (0, 16, 48) for hf in (0, 1)], '(ideal 2)')
