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
//   Sim.Round       oracle_round_compute   random modes: push, pull, push-pull over S_t (main.go:65-89 as rounds),
//                                          with the fault model (EdgeLost: edge_lost) and the stall mode (stall_update)
//   FloodSim.Round  oracle_round_compute   FLOOD, the reference's own algorithm (main.go:65-89): every node forwards
//                                          the values it learned last round to Topology[self] (:72) except their
//                                          first sender (:73-75); dedupe :113; messages = RPCs sent
//   FloodSim (faults) flood_faults_round   one walk per (node, value) down Topology[node] in the message's order,
//                                          head-of-line blocked by a lost attempt, stuck for good once StallRounds
//                                          lost attempts expired the neighbour's context (main.go:72-87)
//   AESim.Round     ae_round               gossip_oracle.c:355 (version-vector max-merge, Philox churn)
//
// Status in this image: no Go toolchain exists here or on the GPU box, so this
// package has not been compiled or run ("go test" in this directory checks it
// against tests/golden/golden.json, the fixtures the C oracle and the HIP
// engine are tested against).
package gossipref

import (
	"math/bits"
	"sort"
)

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

// EdgeLost: the edge n -> p (slot j of initiator n) of round t is lost, both
// directions, when a partition (nodes split into parts contiguous blocks) separates
// its ends or its loss draw Philox({n, t, 4, j/4})[j%4] is below loss (DESIGN.md §2.8).
func EdgeLost(seed, N uint64, loss, parts, n, p, t, j uint32) bool {
	if parts > 1 && (uint64(n)*uint64(parts))/N != (uint64(p)*uint64(parts))/N {
		return true
	}
	if loss != 0 {
		x := Philox4x32_10([4]uint32{n, t, 4, j >> 2}, Key(seed))
		if x[j&3] < loss {
			return true
		}
	}
	return false
}

func popcount(x uint64) uint64 { return uint64(bits.OnesCount64(x)) }

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
	// fault model (SetFaults): edge loss threshold, partitions, stall deadline (DESIGN.md §2.8-2.9)
	Loss, Parts, StallRounds uint32
	streak                   []uint8 // lost-exchange streak per node (stall mode)
}

// SetFaults sets the fault model of the rounds that follow; stallRounds > 0 turns on the
// stall mode (a node whose exchanges were lost in stallRounds rounds in a row initiates
// none until the simulation is rebuilt: the reference's expired 2 s context, main.go:77-87).
func (s *Sim) SetFaults(loss, parts, stallRounds uint32) {
	s.Loss, s.Parts, s.StallRounds = loss, parts, stallRounds
	if stallRounds > 0 && s.streak == nil {
		s.streak = make([]uint8, s.N)
	}
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
		stalled := s.StallRounds > 0 && uint32(s.streak[n]) >= s.StallRounds
		lostAny := false
		for j := uint32(0); j < s.K; j++ {
			if j&3 == 0 {
				x = Philox4x32_10([4]uint32{uint32(n), s.T, 0, j >> 2}, key)
			}
			p := uint64(PeerFromWord(x[j&3], s.N, uint32(n)))
			if EdgeLost(s.Seed, s.N, s.Loss, s.Parts, uint32(n), uint32(p), s.T, j) {
				lostAny = true
				continue
			}
			if stalled { // a stalled node initiates nothing; it still answers and receives
				continue
			}
			for w := uint32(0); w < s.W; w++ {
				if pull {
					next[w][n] |= s.S[w][p]
				}
				if push {
					next[w][p] |= s.S[w][n]
				}
			}
		}
		if s.StallRounds > 0 && !stalled { // only n's own streak depends on n's own edges
			if lostAny {
				s.streak[n]++
			} else {
				s.streak[n] = 0
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

// FloodSim is FLOOD over a harness topology (the reference's own algorithm, main.go:65-89).
type FloodSim struct {
	N        uint64
	R, W     uint32
	T        uint32
	Seed     uint64
	Loss     uint32 // faults (NewFloodSim with any of them on: per-edge retries, DESIGN.md §2.9)
	Parts    uint32
	Stall    uint32
	adj      [][]uint32 // Topology[u] as a sorted set
	rows     [][]uint32 // Topology[u] as the message lists it (the walks, faults on)
	row0     []uint64   // CSR start of u's out-edges
	inSrc    [][]uint32 // in-neighbours of v, ascending
	S, Sprev [][]uint64 // [W][N]
	skip     [][]uint64 // fault-free: values whose first sender is in Adj(v)
	faults   bool
	cur, snd [][]uint32 // faults: [R][N] walk position, first sender (walkNone: a client)
	att      [][]uint8  // faults: [R][N] lost attempts at the walk's position
	full     []uint64
}

// NewFloodSim builds the topology (rows as sets, main.go:132-149 / DESIGN.md §2.4).
func NewFloodSim(N uint64, R uint32, adj [][]uint32, seed uint64, loss, parts, stall uint32) *FloodSim {
	W := (R + 63) / 64
	f := &FloodSim{N: N, R: R, W: W, Seed: seed, Loss: loss, Parts: parts, Stall: stall}
	f.faults = loss != 0 || parts > 1 || stall != 0
	f.adj = make([][]uint32, N)
	f.row0 = make([]uint64, N+1)
	f.inSrc = make([][]uint32, N)
	f.rows = make([][]uint32, N)
	var E uint64
	for u := uint64(0); u < N; u++ {
		f.rows[u] = append([]uint32(nil), adj[u]...)
		row := append([]uint32(nil), adj[u]...)
		sort.Slice(row, func(a, b int) bool { return row[a] < row[b] })
		var set []uint32
		for i, v := range row {
			if i == 0 || v != row[i-1] {
				set = append(set, v)
			}
		}
		f.adj[u] = set
		f.row0[u] = E
		E += uint64(len(set))
	}
	f.row0[N] = E
	for u := uint64(0); u < N; u++ { // ascending u: every in-list sorted
		for _, v := range f.adj[u] {
			f.inSrc[v] = append(f.inSrc[v], uint32(u))
		}
	}
	f.S, f.Sprev, f.skip = make([][]uint64, W), make([][]uint64, W), make([][]uint64, W)
	f.full = make([]uint64, W)
	for w := uint32(0); w < W; w++ {
		f.S[w], f.Sprev[w], f.skip[w] = make([]uint64, N), make([]uint64, N), make([]uint64, N)
		if b := R - 64*w; b >= 64 {
			f.full[w] = ^uint64(0)
		} else {
			f.full[w] = (uint64(1) << b) - 1
		}
	}
	f.cur, f.snd, f.att = make([][]uint32, R), make([][]uint32, R), make([][]uint8, R)
	for x := uint32(0); x < R; x++ {
		f.cur[x], f.snd[x], f.att[x] = make([]uint32, N), make([]uint32, N), make([]uint8, N)
		for n := range f.snd[x] {
			f.cur[x][n], f.snd[x][n] = walkNone, walkNone
		}
	}
	return f
}

const walkNone = ^uint32(0)

// Inject is a client broadcast (main.go:102-117); with faults a new value's walk starts next round.
func (f *FloodSim) Inject(n uint64, r uint32) {
	if f.faults && !holds(f.S, n, r) {
		f.cur[r][n], f.att[r][n], f.snd[r][n] = 0, 0, walkNone
	}
	f.S[r/64][n] |= uint64(1) << (r % 64)
}

func holds(S [][]uint64, n uint64, x uint32) bool { return (S[x/64][n]>>(x%64))&1 == 1 }

func contains(row []uint32, x uint32) (int, bool) {
	i := sort.Search(len(row), func(i int) bool { return row[i] >= x })
	return i, i < len(row) && row[i] == x
}

// lost: the message of value x from u to w (position j of u's row) is lost — one SyncRPC per
// value (main.go:81), so one loss draw per message: Philox({u, t, 4 | x<<16, j/4})[j%4].
func (f *FloodSim) lost(u, w uint32, j uint64, x uint32) bool {
	if f.Parts > 1 && (uint64(u)*uint64(f.Parts))/f.N != (uint64(w)*uint64(f.Parts))/f.N {
		return true
	}
	if f.Loss != 0 {
		d := Philox4x32_10([4]uint32{u, f.T, 4 | x<<16, uint32(j >> 2)}, Key(f.Seed))
		if d[j&3] < f.Loss {
			return true
		}
	}
	return false
}

// Round: one synchronous FLOOD round.
func (f *FloodSim) Round() RoundStats {
	N := f.N
	next := make([][]uint64, f.W)
	for w := range next {
		next[w] = append([]uint64(nil), f.S[w]...)
	}
	var msgs uint64
	if !f.faults {
		for v := uint64(0); v < N; v++ {
			deg := uint64(len(f.adj[v]))
			for w := uint32(0); w < f.W; w++ {
				fv := f.S[w][v] &^ f.Sprev[w][v]
				msgs += popcount(fv)*deg - popcount(fv&f.skip[w][v])
				acc := f.S[w][v]
				for _, u := range f.inSrc[v] {
					acc |= f.S[w][u] &^ f.Sprev[w][u]
				}
				nw := acc &^ f.S[w][v]
				var seen, sk uint64
				for _, u := range f.inSrc[v] {
					if seen == nw {
						break
					}
					c := (f.S[w][u] &^ f.Sprev[w][u]) & nw &^ seen
					if _, in := contains(f.adj[v], u); c != 0 && in {
						sk |= c // sender skip, main.go:73
					}
					seen |= c
				}
				next[w][v] = acc
				f.skip[w][v] = sk
			}
		}
	} else {
		// the walks (flood_faults_round): position c of u's row, the sender skipped (main.go:73), a
		// lost attempt holds the later neighbours back, an expired context never moves on
		for u := uint64(0); u < N; u++ {
			row := f.rows[u]
			for x := uint32(0); x < f.R; x++ {
				if !holds(f.S, u, x) {
					continue
				}
				c, a, snd := f.cur[x][u], uint32(f.att[x][u]), f.snd[x][u]
				for c < uint32(len(row)) {
					w := row[c]
					if w == snd {
						c++
						continue
					}
					msgs++
					if f.lost(uint32(u), w, uint64(c), x) {
						if a < 255 {
							a++
						}
						break
					}
					if !holds(f.S, uint64(w), x) {
						next[x/64][w] |= uint64(1) << (x % 64)
						if uint32(u) < f.snd[x][w] {
							f.snd[x][w] = uint32(u)
						}
					}
					if f.Stall != 0 && a >= f.Stall {
						break
					}
					c++
					a = 0
				}
				f.cur[x][u], f.att[x][u] = c, uint8(a)
			}
		}
		for x := uint32(0); x < f.R; x++ { // values learned this round: walks start next round
			for w := uint64(0); w < N; w++ {
				if holds(next, w, x) && !holds(f.S, w, x) {
					f.cur[x][w], f.att[x][w] = 0, 0
				}
			}
		}
	}
	f.Sprev, f.S = f.S, next
	st := RoundStats{Round: f.T, Alive: N, Messages: msgs, Infected: make([]uint64, f.R)}
	for n := uint64(0); n < N; n++ {
		isFull := true
		for w := uint32(0); w < f.W; w++ {
			x := f.S[w][n]
			if x&f.full[w] != f.full[w] {
				isFull = false
			}
			if x != 0 {
				st.Hash += Mix64(x + (uint64(w)*N+n)*gold64)
			}
			for b := uint32(0); b < 64 && 64*w+b < f.R; b++ {
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
	f.T++
	return st
}

// Run rounds until converged, or a round that sends nothing (quiescence), or maxRounds.
func (f *FloodSim) Run(maxRounds int) []RoundStats {
	var out []RoundStats
	for i := 0; i < maxRounds; i++ {
		st := f.Round()
		out = append(out, st)
		if st.Converged || st.Messages == 0 {
			break
		}
	}
	return out
}

// Read is the read handler (main.go:123-130): the slots node n holds.
func (f *FloodSim) Read(n uint64) []uint32 {
	var out []uint32
	for r := uint32(0); r < f.R; r++ {
		if (f.S[r/64][n]>>(r%64))&1 == 1 {
			out = append(out, r)
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

// Round: churn (the spare word of the first peer draw, Philox({n, t, 0, 0})[3], while
// Fanout <= 3; else Philox({n, t, 1, 0})[0]), then every exchange (n, p_j(n, t)) with both
// ends alive merges both S_t rows into both S_{t+1} rows.
func (a *AESim) Round() RoundStats {
	key := Key(a.Seed)
	N, K := a.N, uint64(a.K)
	alive := make([]bool, N)
	for n := uint64(0); n < N; n++ {
		w := Philox4x32_10([4]uint32{uint32(n), a.T, 0, 0}, key)[3]
		if a.Fanout > 3 {
			w = Philox4x32_10([4]uint32{uint32(n), a.T, 1, 0}, key)[0]
		}
		if a.Alive[n] {
			alive[n] = !(w < a.Fail)
		} else {
			alive[n] = w < a.Rec
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
