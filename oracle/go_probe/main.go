// go_probe pins the oracle's one unpinned assumption (A1, SURVEY.md §8c) against the real
// third-party code the reference chunker uses.  It is not run in this repository (the image
// has no Go toolchain); a maintainer with Go 1.16 and the module cache runs
//
//	cd oracle/go_probe && go run . > out.txt
//	diff out.txt expected_int63.txt    # the oracle's A1: T[i] = uint64(rand.Int63())
//	diff out.txt expected_uint64.txt   # the alternative:  T[i] = rand.Uint64()
//
// and exactly one diff is empty: that variant is what GenerateHashes draws.  Both expected
// files are written by the oracle (oracle/go_probe/expected.py, checked in the CPU suite).
//
// What it prints:
//   - table SEED I HEX: buzhash64.GenerateHashes(SEED)[I] (called at chunk/option.go:54);
//   - per case, every segment of every file (one annotation per file, writer.go:118-130) as
//     chunk.Writer.roll cuts it (writer.go:163-189, the same loop over buzhash64 Roll/Sum64),
//     with its DataRef hash BLAKE2b-256 (pachhash/hash.go:27-30):
//     seg FILE OFFSET SIZE CUT HASH.
// The input bytes are the repository's synthetic generator (pfs_amd.cdc.synthetic_bytes):
// word k of file f is splitmix64-finalize((f<<40 | k) + (seed+1)*0x9E3779B97F4A7C15), little
// endian.  The cases are tests/golden/golden.json's first two.
package main

import (
	"bufio"
	"encoding/binary"
	"fmt"
	"os"

	"github.com/chmduquesne/rollinghash/buzhash64"
	"golang.org/x/crypto/blake2b"
)

func synth(offs []uint64, seed uint64) []byte {
	out := make([]byte, offs[len(offs)-1])
	gamma := (seed + 1) * 0x9E3779B97F4A7C15
	var w [8]byte
	for f := 0; f+1 < len(offs); f++ {
		a, b := offs[f], offs[f+1]
		for k := uint64(0); a+8*k < b; k++ {
			z := (uint64(f)<<40 | k) + gamma
			z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9
			z = (z ^ (z >> 27)) * 0x94D049BB133111EB
			z ^= z >> 31
			binary.LittleEndian.PutUint64(w[:], z)
			copy(out[a+8*k:b], w[:])
		}
	}
	return out
}

type params struct {
	bits     uint
	seed     int64
	min, max int
}

// roll is chunk.Writer.roll for one annotation's bytes, from a fresh hash (Annotate and every
// createChunk call resetHash: Reset, then Write of the 64-byte zero window, writer.go:100-103).
func roll(p params, data []byte, emit func(off, size int, cut bool)) {
	h := buzhash64.NewFromUint64Array(buzhash64.GenerateHashes(p.seed))
	reset := func() {
		h.Reset()
		h.Write(make([]byte, 64))
	}
	reset()
	mask := uint64(1)<<p.bits - 1
	start := 0 // the open segment's first byte: numChunkBytesAnnotation = i + 1 - start
	for i, b := range data {
		h.Roll(b)
		seglen := i + 1 - start
		if h.Sum64()&mask == 0 {
			if seglen < p.min {
				continue
			}
			emit(start, seglen, true)
			start = i + 1
			reset()
			continue
		}
		if seglen >= p.max {
			emit(start, seglen, true)
			start = i + 1
			reset()
		}
	}
	if start < len(data) { // the open tail: a DataRef of the file's last chunk piece
		emit(start, len(data)-start, false)
	}
}

func main() {
	out := bufio.NewWriter(os.Stdout)
	defer out.Flush()
	for _, seed := range []int64{0, 1, 2} {
		t := buzhash64.GenerateHashes(seed)
		for _, i := range []int{0, 1, 2, 3, 255} {
			fmt.Fprintf(out, "table %d %d %016x\n", seed, i, t[i])
		}
	}
	cases := []struct {
		name string
		p    params
		seed uint64
		lens []uint64
	}{
		{"small_multi_literal", params{12, 1, 2000, 30000}, 1, smallLens},
		{"c2_mini_8x4MiB", params{23, 1, 1000000, 20000000}, 0xC2,
			[]uint64{4 << 20, 4 << 20, 4 << 20, 4 << 20, 4 << 20, 4 << 20, 4 << 20, 4 << 20}},
	}
	for _, c := range cases {
		offs := make([]uint64, len(c.lens)+1)
		for i, n := range c.lens {
			offs[i+1] = offs[i] + n
		}
		data := synth(offs, c.seed)
		fmt.Fprintf(out, "case %s\n", c.name)
		for f := 0; f < len(c.lens); f++ {
			file := data[offs[f]:offs[f+1]]
			roll(c.p, file, func(off, size int, cut bool) {
				sum := blake2b.Sum256(file[off : off+size])
				k := 0
				if cut {
					k = 1
				}
				fmt.Fprintf(out, "seg %d %d %d %d %x\n", f, off, size, k, sum)
			})
		}
	}
}
