"""Constants of the reference's config.py (config.py:1-22)."""
grid_size = 20

# Stored as BGR! (config.py:4-18) -- used only by debug drawing
penalty_colour_gradient = {
    1.0000: (0, 0, 255),
    0.9166: (0, 60, 255),
    0.8333: (0, 88, 255),
    0.7500: (0, 109, 255),
    0.6666: (0, 128, 255),
    0.5833: (8, 145, 255),
    0.5000: (0, 163, 249),
    0.4166: (0, 183, 232),
    0.3333: (0, 202, 208),
    0.1666: (0, 221, 176),
    0.0833: (0, 239, 129),
    0.0000: (0, 255, 15),
}

close_grid_colour = (255, 187, 111)
mid_grid_colour = (255, 53, 0)
far_grid_colour = (255, 0, 97)
