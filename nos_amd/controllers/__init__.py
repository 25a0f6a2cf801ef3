"""nos_amd.controllers."""
