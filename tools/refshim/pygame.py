"""Empty stand-in: the reference imports pygame only for render_mode='human'."""
