"""avenir_amd.cli"""
