module pfsamd/goprobe

go 1.16

// The versions the reference pins (/root/reference/go.mod:13,75).
require (
	github.com/chmduquesne/rollinghash v4.0.0+incompatible
	golang.org/x/crypto v0.0.0-20201208171446-5f87f3452ae9
)
