"""gfx950 device-side components: K1 probe runner, K2 synthetic loads, PMC device counting."""
