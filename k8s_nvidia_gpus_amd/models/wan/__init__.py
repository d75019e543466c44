"""Wan2.1 text-to-video model family (DiT + umT5 + causal 3-D VAE + flow samplers), MI355X layout."""
