"""Reference-signature recommendation metrics (reference metrics/), computed on the GPU."""
