// Package gossipref is the Go restatement of the engine's round model — the
// "Go reference path with the same Philox seeds" of SURVEY.md §8(c) — so that
// the reference repository (Go, main.go) can check the MI355X engine against
// Go code of its own.  TEST INFRASTRUCTURE: it is the checker, never the
// product path.
//
// It follows oracle/gossip_oracle.c function by function (file:line there):
//   Philox4x32_10   oracle_philox4x32_10   gossip_oracle.c:56  (Random123 / rocRAND philox4x32_10.h:270-302)
//   PeerFromWord    peer_from_word         gossip_oracle.c:74  (replaces Topology[node.ID()], main.go:72)
//   Origin          oracle_origin          gossip_oracle.c:104 (Philox stream tag 2)
//   Mix64           oracle_mix64           gossip_oracle.c:112 (state hash term)
//   Sim.Round       oracle_round_compute   random modes: push, pull, push-pull over S_t (main.go:65-89 as rounds)
//   AESim.Round     ae_round               gossip_oracle.c:355 (version-vector max-merge, Philox churn tag 1)
// FLOOD (the topology flood of main.go:65-89 with its sender skip) and the
// fault model are pinned by the C oracle and the Python property tests only.
//
// Status in this image: no Go toolchain exists here or on the GPU box, so this
// package has not been compiled or run ("go test" in this directory checks it
// against tests/golden/golden.json, the fixtures the C oracle and the HIP
// engine are tested against).
package gossipref

// Philox4x32_10 is the counter-based generator every random choice is drawn from.
func Philox4x32_10(ctr [4]uint32, key [2]uint32) [4]uint32 {
	c0, c1, c2, c3 := ctr[0], ctr[1], ctr[2], ctr[3]
	k0, k1 := key[0], key[1]
	for i := 0; i < 10; i++ {
		m0 := uint64(0xD2511F53) * uint64(c0)
		m1 := uint64(0xCD9E8D57) * uint64(c2)
		n0 := uint32(m1>>32) ^ c1 ^ k0
		n1 := uint32(m1)
		n2 := uint32(m0>>32) ^ c3 ^ k1
		n3 := uint32(m0)
		c0, c1, c2, c3 = n0, n1, n2, n3
		k0 += 0x9E3779B9
		k1 += 0xBB67AE85
	}
	return [4]uint32{c0, c1, c2, c3}
}

// Key splits a 64-bit seed into the Philox key (low word first).
func Key(seed uint64) [2]uint32 { return [2]uint32{uint32(seed), uint32(seed >> 32)} }

// PeerFromWord maps one Philox word to a peer uniform over [0, N) \ {n}.
func PeerFromWord(x uint32, N uint64, n uint32) uint32 {
	p := uint32((uint64(x) * (N - 1)) >> 32)
	if p >= n {
		p++
	}
	return p
}

// Peer is p_j(n, t): counter {n, t, 0, j/4}, word j%4.
func Peer(seed, N uint64, n, t, j uint32) uint32 {
	x := Philox4x32_10([4]uint32{n, t, 0, j >> 2}, Key(seed))
	return PeerFromWord(x[j&3], N, n)
}

// Origin is rumor r's origin node (Philox tag 2).
func Origin(seed, N uint64, r uint32) uint32 {
	x := Philox4x32_10([4]uint32{r, 0, 2, 0}, Key(seed))
	return uint32((uint64(x[0]) * N) >> 32)
}

const gold64 = 0x9E3779B97F4A7C15

// Mix64 is the splitmix64 finalizer used by the state hash.
func Mix64(z uint64) uint64 {
	z ^= z >> 30
	z *= 0xBF58476D1CE4E5B9
	z ^= z >> 27
	z *= 0x94D049BB133111EB
	z ^= z >> 31
	return z
}

// RoundStats are the per-round observables the engine reports (gossip_round_stats_t).
type RoundStats struct {
	Round     uint32
	Full      uint64
	Alive     uint64
	Converged bool
	Messages  uint64
	Hash      uint64
	Infected  []uint64
}

// Mode of a random-peer simulation.
const (
	Push     = 1
	Pull     = 2
	PushPull = 3
)

// Sim holds N nodes x R rumors as W = ceil(R/64) words per node, word w of
// node n at S[w][n] (the engine's structure-of-arrays layout).
type Sim struct {
	N    uint64
	R, W uint32
	Mode int
	K    uint32 // fanout
	Seed uint64
	T    uint32
	S    [][]uint64
	full []uint64 // per word: the bits of the rumors that exist
}

// NewSim is gossip_create for one shard on the CPU.
func NewSim(N uint64, R uint32, mode int, k uint32, seed uint64) *Sim {
	W := (R + 63) / 64
	s := &Sim{N: N, R: R, W: W, Mode: mode, K: k, Seed: seed}
	s.S = make([][]uint64, W)
	s.full = make([]uint64, W)
	for w := uint32(0); w < W; w++ {
		s.S[w] = make([]uint64, N)
		bits := R - 64*w
		if bits >= 64 {
			s.full[w] = ^uint64(0)
		} else {
			s.full[w] = (uint64(1) << bits) - 1
		}
	}
	return s
}

// Inject is a client broadcast of rumor r at node n (broadcast handler, main.go:102-117).
func (s *Sim) Inject(n uint64, r uint32) { s.S[r/64][n] |= uint64(1) << (r % 64) }

// InjectRandom injects every rumor at its Philox origin.
func (s *Sim) InjectRandom() {
	for r := uint32(0); r < s.R; r++ {
		s.Inject(uint64(Origin(s.Seed, s.N, r)), r)
	}
}

// Round runs one synchronous round: every read is of S_t, every write goes to S_{t+1}.
func (s *Sim) Round() RoundStats {
	key := Key(s.Seed)
	next := make([][]uint64, s.W)
	for w := range next {
		next[w] = append([]uint64(nil), s.S[w]...)
	}
	pull := s.Mode == Pull || s.Mode == PushPull
	push := s.Mode == Push || s.Mode == PushPull
	for n := uint64(0); n < s.N; n++ {
		var x [4]uint32
		for j := uint32(0); j < s.K; j++ {
			if j&3 == 0 {
				x = Philox4x32_10([4]uint32{uint32(n), s.T, 0, j >> 2}, key)
			}
			p := uint64(PeerFromWord(x[j&3], s.N, uint32(n)))
			for w := uint32(0); w < s.W; w++ {
				if pull {
					next[w][n] |= s.S[w][p]
				}
				if push {
					next[w][p] |= s.S[w][n]
				}
			}
		}
	}
	s.S = next
	st := RoundStats{Round: s.T, Alive: s.N, Infected: make([]uint64, s.R)}
	for n := uint64(0); n < s.N; n++ {
		isFull := true
		for w := uint32(0); w < s.W; w++ {
			x := s.S[w][n]
			if x&s.full[w] != s.full[w] {
				isFull = false
			}
			if x != 0 {
				st.Hash += Mix64(x + (uint64(w)*s.N+n)*gold64)
			}
			for b := uint32(0); b < 64 && 64*w+b < s.R; b++ {
				if (x>>b)&1 == 1 {
					st.Infected[64*w+b]++
				}
			}
		}
		if isFull {
			st.Full++
		}
	}
	st.Converged = st.Full == st.Alive
	s.T++
	return st
}

// Run rounds until converged or maxRounds (gossip_step).
func (s *Sim) Run(maxRounds int) []RoundStats {
	var out []RoundStats
	for i := 0; i < maxRounds; i++ {
		st := s.Round()
		out = append(out, st)
		if st.Converged {
			break
		}
	}
	return out
}

// AESim is the anti-entropy mode (configs[4]): K uint32 versions per node,
// push-pull max-merge with k Philox peers among alive nodes, Philox churn.
type AESim struct {
	N          uint64
	K, Fanout  uint32
	Seed       uint64
	Fail, Rec  uint32 // churn thresholds (probability * 2^32)
	T          uint32
	V          []uint32 // V[n*K + c]
	Alive      []bool
	Target     []uint32 // global max vector
}

// NewAESim starts with every node alive and all versions zero.
func NewAESim(N uint64, K, k uint32, seed uint64, fail, rec uint32) *AESim {
	a := &AESim{N: N, K: K, Fanout: k, Seed: seed, Fail: fail, Rec: rec}
	a.V = make([]uint32, N*uint64(K))
	a.Alive = make([]bool, N)
	for i := range a.Alive {
		a.Alive[i] = true
	}
	a.Target = make([]uint32, K)
	return a
}

// InjectRandom sets V[n][c] = Philox({n, c/4, 3, 0})[c%4] & 0xFFFF (oracle_inject_random).
func (a *AESim) InjectRandom() {
	key := Key(a.Seed)
	for c := range a.Target {
		a.Target[c] = 0
	}
	for n := uint64(0); n < a.N; n++ {
		for c := uint32(0); c < a.K; c += 4 {
			x := Philox4x32_10([4]uint32{uint32(n), c >> 2, 3, 0}, key)
			for q := uint32(0); q < 4 && c+q < a.K; q++ {
				v := x[q] & 0xFFFF
				a.V[n*uint64(a.K)+uint64(c+q)] = v
				if v > a.Target[c+q] {
					a.Target[c+q] = v
				}
			}
		}
	}
}

// Inject is a client write: component c of node n gets a newer version.
func (a *AESim) Inject(n uint64, c uint32) {
	i := n*uint64(a.K) + uint64(c)
	a.V[i]++
	if a.V[i] > a.Target[c] {
		a.Target[c] = a.V[i]
	}
}

// Round: churn (Philox tag 1), then every exchange (n, p_j(n, t)) with both
// ends alive merges both S_t rows into both S_{t+1} rows.
func (a *AESim) Round() RoundStats {
	key := Key(a.Seed)
	N, K := a.N, uint64(a.K)
	alive := make([]bool, N)
	for n := uint64(0); n < N; n++ {
		x := Philox4x32_10([4]uint32{uint32(n), a.T, 1, 0}, key)
		if a.Alive[n] {
			alive[n] = !(x[0] < a.Fail)
		} else {
			alive[n] = x[0] < a.Rec
		}
	}
	next := append([]uint32(nil), a.V...)
	st := RoundStats{Round: a.T, Infected: make([]uint64, a.K)}
	for n := uint64(0); n < N; n++ {
		if !alive[n] {
			continue
		}
		var x [4]uint32
		for j := uint32(0); j < a.Fanout; j++ {
			if j&3 == 0 {
				x = Philox4x32_10([4]uint32{uint32(n), a.T, 0, j >> 2}, key)
			}
			p := uint64(PeerFromWord(x[j&3], N, uint32(n)))
			if !alive[p] {
				continue
			}
			st.Messages++
			for c := uint64(0); c < K; c++ {
				u, v := a.V[n*K+c], a.V[p*K+c]
				if v > next[n*K+c] {
					next[n*K+c] = v // pull
				}
				if u > next[p*K+c] {
					next[p*K+c] = u // push
				}
			}
		}
	}
	a.V, a.Alive = next, alive
	for n := uint64(0); n < N; n++ {
		isFull := true
		for c := uint64(0); c < K; c++ {
			v := a.V[n*K+c]
			if v != 0 {
				st.Hash += Mix64(uint64(v) + (c*N+n)*gold64)
			}
			if v != a.Target[c] {
				isFull = false
			} else if alive[n] {
				st.Infected[c]++
			}
		}
		if alive[n] {
			st.Alive++
			if isFull {
				st.Full++
			}
		}
	}
	st.Converged = st.Full == st.Alive
	a.T++
	return st
}

// Run rounds until converged or maxRounds.
func (a *AESim) Run(maxRounds int) []RoundStats {
	var out []RoundStats
	for i := 0; i < maxRounds; i++ {
		st := a.Round()
		out = append(out, st)
		if st.Converged {
			break
		}
	}
	return out
}
