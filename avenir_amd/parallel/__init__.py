"""avenir_amd.parallel"""
