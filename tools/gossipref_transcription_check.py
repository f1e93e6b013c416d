"""Line-by-line Python transcription of oracle/gossipref (Go) Sim.Round (with EdgeLost and the stall
mode), FloodSim.Round (fault-free and per-edge retry paths) and AESim.Round, run on
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


def edge_lost(seed, N, loss, parts, n, p, t, j):  # gossipref.EdgeLost
    if parts > 1 and (n * parts) // N != (p * parts) // N:
        return True
    if loss != 0 and philox([n, t, 4, j >> 2], key(seed))[j & 3] < loss:
        return True
    return False


def msg_lost(seed, N, loss, parts, u, w, t, j, x):  # gossipref.FloodSim.lost
    if parts > 1 and (u * parts) // N != (w * parts) // N:
        return True
    if loss != 0 and philox([u, t, 4 | (x << 16), j >> 2], key(seed))[j & 3] < loss:
        return True
    return False


def random_case(c, max_rounds=256):  # gossipref.Sim (+ SetFaults)
    N, R, k, seed = c["N"], c["R"], c["k"], c["seed"]
    loss, parts, stall = c.get("edge_loss", 0), c.get("partitions", 0), c.get("stall_rounds", 0)
    streak = [0] * N
    W = (R + 63) // 64
    mode = {"push": 1, "pull": 2, "pushpull": 3}[c["mode"]]
    full = [(M64 if R - 64 * w >= 64 else (1 << (R - 64 * w)) - 1) for w in range(W)]
    S = [[0] * N for _ in range(W)]
    inj = [((philox([r, 0, 2, 0], key(seed))[0] * N) >> 32, r) for r in range(R)] if c["inject"] == "random" \
        else c["inject"]
    for n, r in inj:
        S[r // 64][n] |= 1 << (r % 64)
    out = []
    for t in range(max_rounds):
        nx = [row[:] for row in S]
        for n in range(N):
            x = None
            stalled = stall > 0 and streak[n] >= stall
            lost_any = False
            for j in range(k):
                if j & 3 == 0:
                    x = philox([n, t, 0, j >> 2], key(seed))
                p = pfw(x[j & 3], N, n)
                if edge_lost(seed, N, loss, parts, n, p, t, j):
                    lost_any = True
                    continue
                if stalled:
                    continue
                for w in range(W):
                    if mode & 2:
                        nx[w][n] |= S[w][p]
                    if mode & 1:
                        nx[w][p] |= S[w][n]
            if stall > 0 and not stalled:
                streak[n] = streak[n] + 1 if lost_any else 0
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


def pc(x):
    return bin(x).count("1")


def flood_case(c):  # gossipref.FloodSim
    N, R, A = c["N"], c["R"], c["adj"]
    loss, parts, stall = c.get("edge_loss", 0), c.get("partitions", 0), c.get("stall_rounds", 0)
    max_rounds = c.get("max_rounds", 256)
    seed = 0
    W = (R + 63) // 64
    faults = loss != 0 or parts > 1 or stall != 0
    adj = [sorted(set(r)) for r in A]
    row0, E = [], 0
    for u in range(N):
        row0.append(E)
        E += len(adj[u])
    row0.append(E)
    in_src = [[] for _ in range(N)]
    for u in range(N):
        for v in adj[u]:
            in_src[v].append(u)
    rows = [list(r) for r in A]  # faults: Topology[u] as the message lists it
    S = [[0] * N for _ in range(W)]
    Sp = [[0] * N for _ in range(W)]
    skip = [[0] * N for _ in range(W)]
    full = [(M64 if R - 64 * w >= 64 else (1 << (R - 64 * w)) - 1) for w in range(W)]
    NONE = 0xFFFFFFFF
    cur = [[NONE] * N for _ in range(R)]
    snd = [[NONE] * N for _ in range(R)]
    att = [[0] * N for _ in range(R)]

    def holds(X, n, x):
        return (X[x // 64][n] >> (x % 64)) & 1 == 1

    for n, r in c["inject"]:  # FloodSim.Inject
        if faults and not holds(S, n, r):
            cur[r][n], att[r][n], snd[r][n] = 0, 0, NONE
        S[r // 64][n] |= 1 << (r % 64)

    out = []
    for t in range(max_rounds):
        nx = [row[:] for row in S]
        msgs = 0
        if not faults:
            for v in range(N):
                deg = len(adj[v])
                for w in range(W):
                    fv = S[w][v] & ~Sp[w][v] & M64
                    msgs += pc(fv) * deg - pc(fv & skip[w][v])
                    acc = S[w][v]
                    for u in in_src[v]:
                        acc |= S[w][u] & ~Sp[w][u] & M64
                    nw = acc & ~S[w][v] & M64
                    seen = sk = 0
                    for u in in_src[v]:
                        if seen == nw:
                            break
                        cc = (S[w][u] & ~Sp[w][u]) & nw & ~seen & M64
                        if cc and u in adj[v]:
                            sk |= cc
                        seen |= cc
                    nx[w][v] = acc
                    skip[w][v] = sk
        else:
            for u in range(N):
                row = rows[u]
                for x in range(R):
                    if not holds(S, u, x):
                        continue
                    cc, a, sd = cur[x][u], att[x][u], snd[x][u]
                    while cc < len(row):
                        w = row[cc]
                        if w == sd:
                            cc += 1
                            continue
                        msgs += 1
                        if msg_lost(seed, N, loss, parts, u, w, t, cc, x):
                            a = min(a + 1, 255)
                            break
                        if not holds(S, w, x):
                            nx[x // 64][w] |= 1 << (x % 64)
                            snd[x][w] = min(snd[x][w], u)
                        if stall and a >= stall:
                            break
                        cc, a = cc + 1, 0
                    cur[x][u], att[x][u] = cc, a
            for x in range(R):
                for w in range(N):
                    if holds(nx, w, x) and not holds(S, w, x):
                        cur[x][w], att[x][w] = 0, 0
        Sp, S = S, nx
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
        out.append(dict(round=t, full=fc, converged=int(fc == N), messages=msgs, hash=h, infected=inf))
        if fc == N or msgs == 0:
            break
    for node, want in c["reads"].items():
        n = int(node)
        assert [r for r in range(R) if (S[r // 64][n] >> (r % 64)) & 1] == want, (c["name"], node)
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
              ((n, philox([n, t, 0, 0], key(seed))[3] if k <= 3 else philox([n, t, 1, 0], key(seed))[0])
               for n in range(N))]
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
    for c in d["random_faults"]:
        assert random_case(c, c["max_rounds"]) == c["rounds"], c["name"]
        print("ok", c["name"])
    for c in d["flood"] + d["flood_faults"]:
        assert flood_case(c) == c["rounds"], c["name"]
        print("ok", c["name"])
    for c in d["antientropy"]:
        assert ae_case(c) == c["rounds"], c["name"]
        print("ok", c["name"])
