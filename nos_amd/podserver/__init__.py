"""Pod server: many fractional pods per MI355X in one HIP context (MPS analogue)."""
