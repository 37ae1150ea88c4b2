"""avenir_amd.utils"""
