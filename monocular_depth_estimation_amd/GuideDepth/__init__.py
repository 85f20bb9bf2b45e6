"""GuideDepth family (src/GuideDepth/) on MI355X."""
