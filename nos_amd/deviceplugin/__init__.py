"""nos_amd.deviceplugin."""
