"""Drop-in for the reference's match_single_ui.py (match_single_ui.py:20-58): ./UI_use/ in,
./result/UI_disparity/ld{id}.png out, disparity x2.  See match_single.py."""
from .match_single import main_ui

if __name__ == "__main__":
    main_ui()
