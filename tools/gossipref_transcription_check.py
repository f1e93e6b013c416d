"""Line-by-line Python transcription of oracle/gossipref (Go) Sim.Round / AESim.Round, run on
tests/golden/golden.json.  Neither this image nor the GPU box has a Go toolchain, so this is how
the Go restatement's semantics were checked here (the Go test itself: cd oracle/gossipref && go test).
Slow pure-Python loops (about a minute); not part of the pytest suites."""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
d = json.load(open(os.path.join(HERE, "..", "tests", "golden", "golden.json")))
M32, M64, G = 0xFFFFFFFF, (1 << 64) - 1, 0x9E3779B97F4A7C15


def philox(c, k):  # gossipref.Philox4x32_10
    c0, c1, c2, c3 = c
    k0, k1 = k
    for _ in range(10):
        m0, m1 = 0xD2511F53 * c0, 0xCD9E8D57 * c2
        c0, c1, c2, c3 = ((m1 >> 32) ^ c1 ^ k0) & M32, m1 & M32, ((m0 >> 32) ^ c3 ^ k1) & M32, m0 & M32
        k0, k1 = (k0 + 0x9E3779B9) & M32, (k1 + 0xBB67AE85) & M32
    return [c0, c1, c2, c3]


def key(s):
    return [s & M32, (s >> 32) & M32]


def pfw(x, N, n):  # gossipref.PeerFromWord
    p = ((x * (N - 1)) >> 32) & M32
    return p + 1 if p >= n else p


def mix(z):  # gossipref.Mix64
    z &= M64
    z ^= z >> 30
    z = (z * 0xBF58476D1CE4E5B9) & M64
    z ^= z >> 27
    z = (z * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def random_case(c):  # gossipref.Sim
    N, R, k, seed = c["N"], c["R"], c["k"], c["seed"]
    W = (R + 63) // 64
    mode = {"push": 1, "pull": 2, "pushpull": 3}[c["mode"]]
    full = [(M64 if R - 64 * w >= 64 else (1 << (R - 64 * w)) - 1) for w in range(W)]
    S = [[0] * N for _ in range(W)]
    inj = [((philox([r, 0, 2, 0], key(seed))[0] * N) >> 32, r) for r in range(R)] if c["inject"] == "random" \
        else c["inject"]
    for n, r in inj:
        S[r // 64][n] |= 1 << (r % 64)
    out = []
    for t in range(256):
        nx = [row[:] for row in S]
        for n in range(N):
            x = None
            for j in range(k):
                if j & 3 == 0:
                    x = philox([n, t, 0, j >> 2], key(seed))
                p = pfw(x[j & 3], N, n)
                for w in range(W):
                    if mode & 2:
                        nx[w][n] |= S[w][p]
                    if mode & 1:
                        nx[w][p] |= S[w][n]
        S = nx
        h = fc = 0
        inf = [0] * R
        for n in range(N):
            f = True
            for w in range(W):
                x = S[w][n]
                f = f and x & full[w] == full[w]
                if x:
                    h = (h + mix(x + (w * N + n) * G)) & M64
                for b in range(64):
                    if 64 * w + b < R and (x >> b) & 1:
                        inf[64 * w + b] += 1
            fc += f
        out.append(dict(round=t, full=fc, converged=int(fc == N), messages=0, hash=h, infected=inf))
        if fc == N:
            break
    return out


def ae_case(c):  # gossipref.AESim
    N, K, k, seed, fail, rec = c["N"], c["K"], c["k"], c["seed"], c["fail"], c["recover"]
    V, tg, al = [0] * (N * K), [0] * K, [True] * N
    for n in range(N):
        for cc in range(0, K, 4):
            x = philox([n, cc >> 2, 3, 0], key(seed))
            for q in range(4):
                if cc + q < K:
                    V[n * K + cc + q] = x[q] & 0xFFFF
                    tg[cc + q] = max(tg[cc + q], V[n * K + cc + q])
    V[(N - 1) * K] += 1
    tg[0] = max(tg[0], V[(N - 1) * K])
    out = []
    for t in range(300):
        a2 = [(not x < fail) if al[n] else (x < rec) for n, x in
              ((n, philox([n, t, 1, 0], key(seed))[0]) for n in range(N))]
        nx, msgs = V[:], 0
        for n in range(N):
            if not a2[n]:
                continue
            x = None
            for j in range(k):
                if j & 3 == 0:
                    x = philox([n, t, 0, j >> 2], key(seed))
                p = pfw(x[j & 3], N, n)
                if not a2[p]:
                    continue
                msgs += 1
                for cc in range(K):
                    nx[n * K + cc] = max(nx[n * K + cc], V[p * K + cc])
                    nx[p * K + cc] = max(nx[p * K + cc], V[n * K + cc])
        V, al = nx, a2
        h = fc = ac = 0
        inf = [0] * K
        for n in range(N):
            f = True
            for cc in range(K):
                v = V[n * K + cc]
                if v:
                    h = (h + mix(v + (cc * N + n) * G)) & M64
                if v != tg[cc]:
                    f = False
                elif al[n]:
                    inf[cc] += 1
            if al[n]:
                ac += 1
                fc += f
        out.append(dict(round=t, full=fc, alive=ac, converged=int(fc == ac), messages=msgs, hash=h, infected=inf))
        if fc == ac:
            break
    assert V[:K] == c["node0"] and al[0] == c["node0_alive"], c["name"]
    return out


if __name__ == "__main__":
    for v in d["philox_kat"]:
        assert philox(v["ctr"], v["key"]) == v["out"]
    for c in d["random"]:
        assert random_case(c) == c["rounds"], c["name"]
        print("ok", c["name"])
    for c in d["antientropy"]:
        assert ae_case(c) == c["rounds"], c["name"]
        print("ok", c["name"])
