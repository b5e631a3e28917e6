module github.com/eazy-mi355x/eazy

go 1.21
